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
    ap.add_argument("--gaps", type=int, default=12, help="idle time by (kernel before, kernel after) pair")
    ap.add_argument("--timeline", type=int, default=2, help="kernels around the largest gaps (this many gaps)")
    ap.add_argument("--copies", default="", help="rocprofv3 memory_copy_trace.csv: copies shown in the timeline")
    ap.add_argument("--phase-ms", type=float, default=0.0,
                    help="the same phase's wall time measured without the profiler (GPU events)")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    gaps = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]), b) for a, b in zip(idx, idx[1:])]
    i0 = max(gaps)[1] if gaps else idx[0]
    t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[idx[-1]]["End_Timestamp"])
    seg = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
    iv = sorted((int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t1), r["Kernel_Name"]) for r in seg)
    busy, cs, ce, last = 0, iv[0][0], iv[0][1], iv[0][2]
    idle = collections.defaultdict(lambda: [0, 0])
    hist = collections.Counter()
    for a, b, name in iv[1:]:
        if a > ce:
            busy += ce - cs
            g = a - ce
            key = f"{short(last)} -> {short(name)}"
            idle[key][0] += 1
            idle[key][1] += g
            hist[min(g // 10000, 10)] += g
            cs, ce = a, b
        else:
            ce = max(ce, b)
        if b >= ce:
            last = name
    busy += ce - cs
    print(f"phase {(t1 - t0) / 1e6:.1f} ms, {len(seg)} kernels, GPU busy (union) {busy / 1e6:.1f} ms "
          f"({100.0 * busy / max(t1 - t0, 1):.0f} %)")
    if args.phase_ms > 0:
        print(f"unprofiled phase {args.phase_ms:.1f} ms (GPU events): kernel union / unprofiled phase "
              f"{100.0 * busy / 1e6 / args.phase_ms:.0f} % (the kernel trace itself adds per-dispatch gaps)")
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        c[r["Kernel_Name"][:100]][0] += 1
        c[r["Kernel_Name"][:100]][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, (n, t) in sorted(c.items(), key=lambda x: -x[1][1])[:args.top]:
        print(f"{t / 1e6:9.1f} ms {n:6d}  {name}")
    if args.timeline:
        seq = sorted(seg, key=lambda r: int(r["Start_Timestamp"]))
        cps = []
        if args.copies:
            for r in csv.DictReader(open(args.copies)):
                if t0 <= int(r["Start_Timestamp"]) <= t1:
                    cps.append({"Kernel_Name": "COPY " + r.get("Direction", r.get("Kind", "?")),
                                "Start_Timestamp": r["Start_Timestamp"], "End_Timestamp": r["End_Timestamp"]})
        big = sorted(range(1, len(seq)), key=lambda i: -(int(seq[i]["Start_Timestamp"]) -
                                                           max(int(r["End_Timestamp"]) for r in seq[max(0, i - 4):i])))
        for i in sorted(big[:args.timeline]):
            base = int(seq[i]["Start_Timestamp"])
            print(f"timeline around kernel {i} (us relative to its start):")
            lo, hi = int(seq[max(0, i - 14)]["Start_Timestamp"]), int(seq[min(len(seq) - 1, i + 8)]["Start_Timestamp"])
            near = [c for c in cps if lo <= int(c["Start_Timestamp"]) <= hi]
            for r in sorted(seq[max(0, i - 14):i + 8] + near, key=lambda r: int(r["Start_Timestamp"])):
                a, b = int(r["Start_Timestamp"]) - base, int(r["End_Timestamp"]) - base
                print(f"   {a / 1e3:9.1f} {b / 1e3:9.1f}  {short(r['Kernel_Name'])}")
    if args.gaps:
        print("idle by gap length (10 us buckets, last = 100 us and more):",
              " ".join(f"{10 * k}+:{hist[k] / 1e6:.1f}ms" for k in sorted(hist)))
        print("idle by the kernels around the gap:")
        for key, (n, t) in sorted(idle.items(), key=lambda x: -x[1][1])[:args.gaps]:
            print(f"{t / 1e6:9.2f} ms {n:6d}  {key}")


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name.split("::")[-1][:48]


if __name__ == "__main__":
    main()
