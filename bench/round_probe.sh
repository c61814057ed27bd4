#!/bin/bash
# Work-item statistics plus a per-round kernel timeline of GBDT at 10M rows (GPU box).
# Usage: [EXTRA="--tail-words 1000000"] bash bench/round_probe.sh <tag> [trees]
set -e
TAG=${1:-probe}
TREES=${2:-12}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${ITEMS:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench/item_stats.py --rows 10000000 > "$OUT/items.txt" 2>&1
  cat "$OUT/items.txt"
fi
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/gbdt_train.py --rows 10000000 --trees "$TREES" $EXTRA > "$OUT/prof.log" 2>&1
T=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python bench/trace_rounds.py "$T" --round 6 --sequence > "$OUT/rounds.txt"
head -60 "$OUT/rounds.txt"
rm -f "$T"
