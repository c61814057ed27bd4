#!/bin/bash
# Host spans (no device sync) of BASELINE config 2's GBDT fit with the runner's C++ level loop on
# and off (FDX_GBDT_CXX_LEVELS): how the fit time splits into prepare / workspace / rounds.
# Usage: bash bench/gbdt_spans_ab.sh <tag>
set -e
TAG=${1:-gspans}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 1 0 1 0; do
  FDX_GBDT_CXX_LEVELS=$v FDX_TRACE=$OUT/g$v.jsonl timeout -k 10 300 python -u bench/suite.py gbdt_1m > "$OUT/g$v.json" 2> "$OUT/g$v.err"
  echo "cxx=$v $(tail -1 "$OUT/g$v.json" | grep -o 'fit_only_s": [0-9.]*')"
  python bench/span_last_fit.py "$OUT/g$v.jsonl" --depth 2 > "$OUT/spans_$v.txt"
  head -14 "$OUT/spans_$v.txt"
  rm -f "$OUT/g$v.jsonl"
done
