#!/bin/bash
# GPU tests, then the 10M-row GBDT timing (20 trees, twice) and a per-round kernel timeline.
# Usage: bash bench/gpu_check.sh <tag>
set -e
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees 20 2>/dev/null | tail -1 | tee -a "$OUT/gbdt20.txt"
done
ITEMS=0 bash bench/round_probe.sh "$TAG/probe" 12 > /dev/null
