#!/bin/bash
# Trees per lockstep batch (FDX_RF_INFLIGHT) on the DP=8 shard (forced collectives) and on 10M
# rows. Usage: bash bench/rf_lanes_sweep.sh <tag> "16 32 48" [rows...]
set -e
TAG=${1:-rfsw}
LANES=${2:-"16 32"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in $LANES; do
  FDX_RF_INFLIGHT=$n FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1 timeout -k 10 300 python -u bench/suite.py rf \
    --rows 1250000 > "$OUT/dp_$n.json" 2> "$OUT/dp_$n.err"
  echo "dp lanes $n $(tail -1 "$OUT/dp_$n.json" | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["train_only_s"], r["lanes"], r["collective_calls"], r["level_collective_ms"], r.get("batch_host_s"))')"
done
