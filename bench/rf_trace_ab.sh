#!/bin/bash
# Kernel traces of RF 500 x depth 5 at 10M rows, preselected lists on / off (rocprofv3 kernel
# trace + stats; GPU busy union via bench/trace_busy.py). Usage: bash bench/rf_trace_ab.sh <tag>
set -e
TAG=${1:-rftr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for PS in 1 0; do
  FDX_RF_PRESELECT=$PS timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$PS" -o run -- \
    python3 bench/suite.py rf > "$OUT/rf_presel$PS.json" 2> "$OUT/rf_presel$PS.err"
  tail -1 "$OUT/rf_presel$PS.json"
  TR=$(find "$OUT/prof$PS" -name "*kernel_trace.csv" | head -1)
  python bench/trace_busy.py "$TR" --marker rf_window_kernel --top 18 > "$OUT/busy_presel$PS.txt"
  cat "$OUT/busy_presel$PS.txt"
  rm -f "$TR"
done
