#!/bin/bash
# RF 500 trees x depth 5 on 10M rows (BASELINE config 3, 1 GPU): preselected item lists (one wave
# per active item) vs the r4 passes. Usage: bash bench/rf_ab.sh <tag>
set -e
TAG=${1:-rfab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for PS in 1 0; do
  FDX_RF_PRESELECT=$PS timeout -k 10 300 python -u bench/suite.py rf > "$OUT/rf10M_presel$PS.json" 2> "$OUT/rf10M_presel$PS.err"
  cat "$OUT/rf10M_presel$PS.json"
done
