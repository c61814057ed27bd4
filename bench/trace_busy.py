"""GPU busy share of a phase in a rocprofv3 kernel trace: the phase runs from the first marker
kernel after the largest gap between marker kernels (the warm-up's markers come earlier) to the
last marker kernel; prints its wall time, the union of all kernels' busy intervals inside it
(concurrent streams counted once) and the top kernels by summed time.

Usage: python bench/trace_busy.py run_kernel_trace.csv --marker rf_window_kernel
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="rf_window_kernel")
    ap.add_argument("--top", type=int, default=15)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    gaps = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]), b) for a, b in zip(idx, idx[1:])]
    i0 = max(gaps)[1] if gaps else idx[0]
    t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[idx[-1]]["End_Timestamp"])
    seg = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
    iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t1)) for r in seg)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    busy += ce - cs
    print(f"phase {(t1 - t0) / 1e6:.1f} ms, {len(seg)} kernels, GPU busy (union) {busy / 1e6:.1f} ms "
          f"({100.0 * busy / max(t1 - t0, 1):.0f} %)")
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        c[r["Kernel_Name"][:100]][0] += 1
        c[r["Kernel_Name"][:100]][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, (n, t) in sorted(c.items(), key=lambda x: -x[1][1])[:args.top]:
        print(f"{t / 1e6:9.1f} ms {n:6d}  {name}")


if __name__ == "__main__":
    main()
