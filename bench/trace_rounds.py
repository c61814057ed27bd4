"""Per-boosting-round breakdown of a rocprofv3 kernel trace (``*_kernel_trace.csv``).

Rounds are delimited by the kernel that starts each GBDT round (``logistic_grad``, or the fused
``grad_max`` of the native level runner). Prints, for a
few rounds, the wall time between round starts, the summed kernel time (GPU busy) and the
per-kernel split of one round.

Usage: python bench/trace_rounds.py gpurun_out/.../run_kernel_trace.csv [--round 6]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--round", type=int, default=6)
    ap.add_argument("--marker", default=None, help="round-start kernel (default: logistic_grad, else grad_max)")
    ap.add_argument("--sequence", action="store_true", help="also list the kernels of the round in order")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    markers = [args.marker] if args.marker else ["logistic_grad", "grad_max_kernel"]
    idx = []
    for m in markers:
        idx = [i for i, r in enumerate(rows) if m in r["Kernel_Name"]]
        if idx:
            break
    if len(idx) < 3:
        print(f"{len(idx)} rounds: too few to split")
        return
    print(f"{len(idx)} rounds")
    for a, b in zip(idx[1:-1], idx[2:]):
        seg = rows[a:b]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        print(f"round wall {(t1 - t0) / 1e6:7.2f} ms  busy {busy / 1e6:7.2f} ms  kernels {len(seg)}")
    k = min(args.round, len(idx) - 2)
    seg = rows[idx[k]:idx[k + 1]]
    c = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        name = r["Kernel_Name"][:110]
        c[name][0] += 1
        c[name][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, (n, t) in sorted(c.items(), key=lambda x: -x[1][1]):
        print(f"{t / 1e6:8.3f} ms {n:4d}  {name}")
    if args.sequence:
        t0 = int(seg[0]["Start_Timestamp"])
        for r in seg:
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(a - t0) / 1e6:8.3f} +{(b - a) / 1e6:7.3f} ms  {r['Kernel_Name'][:100]}")


if __name__ == "__main__":
    main()
