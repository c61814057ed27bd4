#!/bin/bash
# Kernel traces of RF 500 x depth 5 on a 1.25M-row shard with forced collectives, preselected
# item lists on / off: GPU busy union + top kernels. Usage: bash bench/rf_dp_trace_ab.sh <tag>
set -e
TAG=${1:-rfdptrab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1
for PS in 0 1; do
  FDX_RF_PRESELECT=$PS timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$PS" -o run -- \
    python3 bench/suite.py rf --rows 1250000 > "$OUT/rf$PS.json" 2> "$OUT/rf$PS.err"
  TR=$(find "$OUT/prof$PS" -name "*kernel_trace.csv" | head -1)
  python bench/trace_busy.py "$TR" --marker rf_window_kernel --top 16 > "$OUT/busy$PS.txt"
  echo "presel $PS"; cat "$OUT/busy$PS.txt"
  rm -f "$TR"
done
