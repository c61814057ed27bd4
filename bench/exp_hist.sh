#!/bin/bash
# Histogram kernel A/B: rocprofv3 kernel stats of a 10-tree 10M-row GBDT run per environment setting.
# Usage (GPU box, repo root): bash bench/exp_hist.sh <tag> "ENV=a" "ENV=b" ...   ("" = defaults)
set -e
export TMPDIR=/tmp
TAG=${1:-exp}; shift
i=0
for SETTING in "${@:-}"; do
  i=$((i + 1))
  mkdir -p gpurun_out/$TAG$i
  echo "$SETTING" > gpurun_out/$TAG$i/setting
  env $SETTING timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG$i/prof -o run -- python3 bench/gbdt_train.py --rows 10000000 --trees 10 > gpurun_out/$TAG$i/log 2>&1
  echo "$SETTING: $(grep rows gpurun_out/$TAG$i/log)"
done
