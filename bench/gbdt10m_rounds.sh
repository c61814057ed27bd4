#!/bin/bash
# GBDT 100 trees x depth 6 on 10M rows (the bench.py training shape): kernel trace split per
# boosting round (bench/trace_rounds.py), one late round listed kernel by kernel, plus the fit's
# kernel totals. Usage: bash bench/gbdt10m_rounds.sh <tag> [round]
set -e
TAG=${1:-g10m_rounds}
RND=${2:-16}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/gbdt_train.py --rows 10000000 --trees 100 > "$OUT/fit.json" 2> "$OUT/fit.err"
tail -1 "$OUT/fit.json" | cut -c1-400
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python bench/trace_rounds.py "$TR" --round "$RND" --sequence > "$OUT/rounds.txt" 2>&1 || true
ST=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
cp "$ST" "$OUT/kernel_stats.csv"
rm -f "$TR"
