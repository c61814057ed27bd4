"""Sum a FDX_TRACE span log (utils/tracing.py JSONL) by span name: calls, total and mean ms.

Usage: python bench/span_summary.py trace.jsonl [--depth 1]
"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--depth", type=int, default=99, help="only spans at nesting depth <= this")
    ap.add_argument("--last", action="store_true", help="per name, the duration of its LAST call only (a bench's "
                    "timed fit follows its warm-up)")
    args = ap.parse_args()
    tot = collections.defaultdict(lambda: [0, 0.0])
    for line in open(args.trace):
        r = json.loads(line)
        if r.get("depth", 0) > args.depth:
            continue
        key = (r.get("depth", 0), r["name"])
        if args.last:
            tot[key] = [1, r["dur_ms"]]
            continue
        tot[key][0] += 1
        tot[key][1] += r["dur_ms"]
    for (d, name), (n, ms) in sorted(tot.items(), key=lambda x: (-x[1][1])):
        print(f"{'  ' * d}{name:<28s} {n:6d} calls {ms:10.2f} ms  ({ms / n:8.3f} ms each)")


if __name__ == "__main__":
    main()
