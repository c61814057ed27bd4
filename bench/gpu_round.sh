#!/bin/bash
# One GPU-box iteration: tree-engine GPU tests, 10M-row GBDT timing, rocprofv3 kernel stats.
# Usage (on the GPU box, from the repo root): bash bench/gpu_round.sh <tag> [trees]
set -e
TAG=${1:-run}
TREES=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees "$TREES" > "$OUT/plain.json" 2> "$OUT/plain.err"
cat "$OUT/plain.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/gbdt_train.py --rows 10000000 --trees "$TREES" > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -25 {} \; | cut -c1-220
