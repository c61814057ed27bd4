#!/bin/bash
# DP per-rank critical path at shard size: RF 500 trees x depth 5 and
# GBDT 100 trees x depth 6 on a 1.25M-row shard (10M / DP=8) with every collective forced
# through RCCL at world 1 (FDX_FORCE_COLLECTIVES=1). Usage: bash bench/dp_shard.sh <tag>
set -e
TAG=${1:-dp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FDX_FORCE_COLLECTIVES=1
FDX_RF_COMPACT=1 timeout -k 10 300 python -u bench/suite.py rf --rows 1250000 > "$OUT/rf.json" 2> "$OUT/rf.err"
cat "$OUT/rf.json"
timeout -k 10 300 python -u bench/suite.py xgb --rows 1250000 --trees 100 > "$OUT/gbdt.json" 2> "$OUT/gbdt.err"
cat "$OUT/gbdt.json"
