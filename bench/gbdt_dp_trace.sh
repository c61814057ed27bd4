#!/bin/bash
# GBDT 100 x depth 6 on a 1.25M-row shard (10M / DP=8) with every collective forced through RCCL
# at world 1: kernel trace split per boosting round. Usage: bash bench/gbdt_dp_trace.sh <tag>
set -e
TAG=${1:-gdp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export FDX_FORCE_COLLECTIVES=1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/suite.py xgb --rows 1250000 --trees 100 > "$OUT/gbdt.json" 2> "$OUT/gbdt.err"
tail -1 "$OUT/gbdt.json" | cut -c1-300
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python bench/trace_rounds.py "$TR" --round 50 --sequence > "$OUT/rounds.txt" 2>&1 || true
head -12 "$OUT/rounds.txt"; grep -A30 "^round wall" "$OUT/rounds.txt" | grep -v "^round" | head -30
CP=$(find "$OUT/prof" -name "*memory_copy_trace.csv" | head -1)
python bench/trace_busy.py "$TR" --marker grad_max --top 12 --gaps 14 --timeline 1 ${CP:+--copies "$CP"} > "$OUT/busy.txt"
cat "$OUT/busy.txt"
rm -f "$TR" "$CP"
