#!/bin/bash
# Host spans of the DP=8-shard forest (1.25M rows, forced collectives): what train_only_s holds
# besides the level loop. Usage: bash bench/rf_dp_spans.sh <tag>
set -e
TAG=${1:-rfsp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1
FDX_TRACE=$OUT/rf.jsonl timeout -k 10 300 python -u bench/suite.py rf --rows 1250000 > "$OUT/rf.json" 2> "$OUT/rf.err"
tail -1 "$OUT/rf.json" | cut -c1-300
python bench/span_summary.py "$OUT/rf.jsonl" --last > "$OUT/rf_spans_last.txt"
python bench/span_summary.py "$OUT/rf.jsonl" > "$OUT/rf_spans.txt"
head -30 "$OUT/rf_spans_last.txt"
rm -f "$OUT/rf.jsonl"
