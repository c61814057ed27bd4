"""Summarise an ``FDX_TRACE`` span log: total / count / mean wall time per span name.

Usage: python bench/span_summary.py trace.jsonl
"""
import collections
import json
import sys


def main(path):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for line in open(path):
        r = json.loads(line)
        a = agg[r["name"]]
        a[0] += 1
        a[1] += r.get("dur_ms", r.get("ms", 0.0))
    for name, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{t:10.1f} ms {n:7d}  {t / n:8.3f} ms/call  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
