#!/bin/bash
# GBDT training profile on one MI355X: plain timing, synchronised span trace, rocprofv3 kernel stats.
# Usage (on the GPU box, from the repo root): bash bench/prof_gbdt.sh [rows] [trees] [outdir]
set -e
ROWS=${1:-10000000}
TREES=${2:-20}
OUT=${3:-gpurun_out/prof_gbdt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" > "$OUT/plain.json" 2>&1
FDX_TRACE_SYNC=1 timeout -k 10 300 python bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" \
  --trace "$OUT/trace.jsonl" > "$OUT/traced.json" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" > "$OUT/prof.log" 2>&1
