#!/bin/bash
# GBDT 20 trees x depth 6 on 10M rows (the bench.py headline training shape): kernel trace split
# per boosting round (bench/trace_rounds.py), for the default level path and, with a second
# argument, for FDX_NATIVE_LEVELS=0 (the Python-issued level path) as the A/B.
# Usage: bash bench/gbdt10m_trace.sh <tag> [ab]
set -e
TAG=${1:-g10m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {
  local name=$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
    python3 bench/gbdt_train.py --rows 10000000 --trees 20 > "$OUT/$name.json" 2> "$OUT/$name.err"
  tail -1 "$OUT/$name.json" | cut -c1-300
  TR=$(find "$OUT/prof_$name" -name "*kernel_trace.csv" | head -1)
  python bench/trace_rounds.py "$TR" --round 10 > "$OUT/rounds_$name.txt" 2>&1 || true
  head -14 "$OUT/rounds_$name.txt"; sed -n '/^ *[0-9.]* ms  *[0-9]*  /p' "$OUT/rounds_$name.txt" | head -16
  rm -f "$TR"
}
run native
if [ -n "$2" ]; then FDX_NATIVE_LEVELS=0 run python; fi
