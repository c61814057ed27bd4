#!/bin/bash
# A/B one environment knob on the 10M-row GBDT timing (GPU box), after the tree-engine GPU tests.
# Usage: bash bench/ab_env.sh <tag> <trees> "<env A>" "<env B>" [repeats]
set -e
TAG=${1:-ab}
TREES=${2:-20}
A=${3:-}
B=${4:-}
REP=${5:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for i in $(seq "$REP"); do
  for E in "$A" "$B"; do
    echo "== [$E]"
    env $E timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees "$TREES" 2>/dev/null | tail -1
  done
done | tee "$OUT/ab.txt"
