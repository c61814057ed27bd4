#!/bin/bash
# BASELINE config 4 on ONE MI355X: XGBoost-compatible GBDT, 1000 trees x depth 6 on 100M rows
# (the whole dataset of the DP=8 config on a single GPU: the row-capacity check of utils/memory.py).
# A heartbeat line every 30 s keeps the run visibly alive. Usage: bash bench/xgb_config4.sh <tag> [rows] [trees]
set -e
TAG=${1:-xgb4}
ROWS=${2:-100000000}
TREES=${3:-1000}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u bench/suite.py xgb --rows "$ROWS" --trees "$TREES" > "$OUT/xgb.json" 2> "$OUT/xgb.err" &
PID=$!
while kill -0 $PID 2>/dev/null; do sleep 30; echo "alive $(date +%T) $(tail -c 200 "$OUT/xgb.err" | tr '\n' ' ' | cut -c1-150)"; done
wait $PID
tail -1 "$OUT/xgb.json" | cut -c1-900
