#!/bin/bash
# Sweep environment knobs of the GBDT trainer on one GPU: each argument is a space-separated
# list of VAR=VALUE settings; prints one JSON line per setting (bench/gbdt_train.py, 10M rows).
# Usage (GPU box, repo root): TREES=20 bash bench/sweep_env.sh "FDX_DENSE_MAX_DEPTH=2" "FDX_DENSE_MAX_DEPTH=5"
set -e
TREES=${TREES:-20}
ROWS=${ROWS:-10000000}
mkdir -p gpurun_out/sweep
i=0
for setting in "$@"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  env $setting timeout -k 10 200 python bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" \
    > gpurun_out/sweep/s$i.json 2> gpurun_out/sweep/s$i.err
  echo "{\"setting\": \"$setting\", \"result\": $(cat gpurun_out/sweep/s$i.json)}"
done
