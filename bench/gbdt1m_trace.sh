#!/bin/bash
# BASELINE config 2 (GBDT 100 trees x depth 6 on 1M rows, 1 GPU): plain timing, then a kernel
# trace with per-round kernel counts (bench/trace_rounds.py). Usage: bash bench/gbdt1m_trace.sh <tag>
set -e
TAG=${1:-g1m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u bench/suite.py gbdt_1m > "$OUT/gbdt_1m.json" 2> "$OUT/gbdt_1m.err"
tail -1 "$OUT/gbdt_1m.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/suite.py gbdt_1m > "$OUT/prof.log" 2>&1
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python bench/trace_rounds.py "$TR" --sequence > "$OUT/rounds.txt" 2>&1 || true
head -4 "$OUT/rounds.txt"; tail -130 "$OUT/rounds.txt"
rm -f "$TR"
