#!/bin/bash
# RF 500 x depth 5 on a 1.25M-row shard with forced collectives: lanes x groups sweep + a host
# profile of the default. Usage: bash bench/rf_dp_sweep.sh <tag>
set -e
TAG=${1:-rfdp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1
timeout -k 10 200 python -u bench/probes/rf_host_probe.py --rows 1250000 --forced > "$OUT/host_profile.txt" 2> "$OUT/host_profile.err"
head -45 "$OUT/host_profile.txt"
for LG in "16 2" "32 2" "32 4"; do
  set -- $LG
  FDX_RF_INFLIGHT=$1 FDX_RF_GROUPS=$2 timeout -k 10 200 python -u bench/suite.py rf --rows 1250000 > "$OUT/rf_l$1_g$2.json" 2> "$OUT/rf_l$1_g$2.err"
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/rf_l$1_g$2.json') if l.startswith('{')][-1]); print('lanes $1 groups $2', d['train_only_s'], d['collective_calls'], d['level_collective_ms'])"
done
