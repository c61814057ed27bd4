#!/bin/bash
# Kernel trace of RF 500 x depth 5 (BASELINE config 3 shape): GPU busy share of the forest and
# the top kernels. Usage: bash bench/rf_trace.sh <tag> [rows (default 10M)] [forced: 1 = every
# collective through RCCL at world 1, the DP per-rank path]
set -e
TAG=${1:-rftr}
ROWS=${2:-10000000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ "${3:-0}" = "1" ]; then export FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/suite.py rf --rows "$ROWS" > "$OUT/rf.json" 2> "$OUT/rf.err"
tail -1 "$OUT/rf.json" | cut -c1-400
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python bench/trace_busy.py "$TR" --marker rf_window_kernel --top 30 > "$OUT/busy.txt"
cat "$OUT/busy.txt"
rm -f "$TR"
