"""Per-name span totals of the LAST gbdt fit in a FDX_TRACE log (spans starting at or after the
last gbdt.prepare): calls, total ms, mean ms, at nesting depth <= --depth.
Usage: python bench/span_last_fit.py trace.jsonl [--depth 1] [--first prepare-span-name]"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--first", default="gbdt.prepare")
    args = ap.parse_args()
    recs = [json.loads(line) for line in open(args.trace)]
    t0 = max(r["t"] for r in recs if r["name"] == args.first)
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in recs:
        if r["t"] >= t0 and r.get("depth", 0) <= args.depth:
            k = (r.get("depth", 0), r["name"])
            tot[k][0] += 1
            tot[k][1] += r["dur_ms"]
    for (d, name), (n, ms) in sorted(tot.items(), key=lambda x: -x[1][1]):
        print(f"{'  ' * d}{name:<28s} {n:6d} calls {ms:10.2f} ms  ({ms / n:8.3f} ms each)")


if __name__ == "__main__":
    main()
