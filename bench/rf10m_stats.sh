#!/bin/bash
# RandomForest 500 trees x depth 5 on 10M rows (bench/suite.py rf): kernel statistics of the whole
# run (the forest's kernels dominate the trained part). Usage: bash bench/rf10m_stats.sh <tag>
set -e
TAG=${1:-rf10m_stats}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/suite.py rf --rows 10000000 > "$OUT/rf.json" 2> "$OUT/rf.err"
tail -1 "$OUT/rf.json" | cut -c1-300
ST=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
cp "$ST" "$OUT/kernel_stats.csv"
find "$OUT/prof" -name "*kernel_trace.csv" -delete
