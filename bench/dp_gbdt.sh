#!/bin/bash
# GBDT 100 x depth 6 on a 1.25M-row shard (10M / DP=8) with every collective forced through RCCL
# at world 1 (the DP=8 per-rank path on one GPU). Usage: bash bench/dp_gbdt.sh <tag> [extra env]
set -e
TAG=${1:-dpg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FDX_FORCE_COLLECTIVES=1
for i in 1 2; do
  timeout -k 10 300 python -u bench/suite.py xgb --rows 1250000 --trees 100 > "$OUT/gbdt_$i.json" 2> "$OUT/gbdt_$i.err"
  tail -1 "$OUT/gbdt_$i.json" | cut -c1-420
done
