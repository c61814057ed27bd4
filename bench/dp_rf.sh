#!/bin/bash
# RF 500 x depth 5 on a 1.25M-row shard (10M / DP=8) with every collective forced through RCCL at
# world 1 (the DP=8 per-rank path on one GPU), twice. Usage: bash bench/dp_rf.sh <tag>
set -e
TAG=${1:-dpr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1
for i in 1 2; do
  timeout -k 10 300 python -u bench/suite.py rf --rows 1250000 > "$OUT/rf_$i.json" 2> "$OUT/rf_$i.err"
  tail -1 "$OUT/rf_$i.json" | cut -c1-600
done
