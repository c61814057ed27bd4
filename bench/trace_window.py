"""Kernels of a rocprofv3 kernel trace inside a time window around a marker kernel: the setup a
GBDT fit runs before its first boosting round, for example.

Usage: python bench/trace_window.py run_kernel_trace.csv --marker logistic_grad --before-ms 150
Prints per-kernel totals inside [first marker - before_ms, first marker), then the gaps: the
window's wall time minus the union of its kernels' busy intervals (host time between launches).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="logistic_grad")
    ap.add_argument("--before-ms", type=float, default=150.0)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the LAST marker-free stretch before the first marker of the timed fit: the warm-up fit has
    # markers too, so take the first marker after the largest gap between consecutive markers
    idx = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    if not idx:
        raise SystemExit("marker not found")
    gaps = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]), b) for a, b in zip(idx, idx[1:])]
    first = max(gaps)[1] if gaps else idx[0]
    t1 = int(rows[first]["Start_Timestamp"])
    t0 = t1 - int(args.before_ms * 1e6)
    seg = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    c = collections.defaultdict(lambda: [0, 0])
    iv = []
    for r in seg:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c[r["Kernel_Name"][:100]][0] += 1
        c[r["Kernel_Name"][:100]][1] += b - a
        iv.append((a, b))
    iv.sort()
    busy, cs, ce = 0, None, None
    for a, b in iv:
        if cs is None:
            cs, ce = a, b
        elif a > ce:
            busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if cs is not None:
        busy += ce - cs
    print(f"window {args.before_ms:.1f} ms before the timed fit's first {args.marker}: {len(seg)} kernels, "
          f"busy {busy / 1e6:.2f} ms")
    for name, (n, t) in sorted(c.items(), key=lambda x: -x[1][1])[:args.top]:
        print(f"{t / 1e6:9.3f} ms {n:5d}  {name}")


if __name__ == "__main__":
    main()
