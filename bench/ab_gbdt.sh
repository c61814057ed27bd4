#!/bin/bash
# A/B(/C...) timing of GBDT training on one MI355X under several environment settings (each run
# twice, interleaved), then a rocprofv3 kernel-stats run of the last setting.
# Usage (GPU box, repo root):
#   ROWS=10000000 TREES=20 OUT=gpurun_out/ab bash bench/ab_gbdt.sh "FDX_HIST_SRC=stream" "FDX_HIST_SRC=record"
set -e
ROWS=${ROWS:-10000000}
TREES=${TREES:-20}
OUT=${OUT:-gpurun_out/ab_gbdt}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    env $setting timeout -k 10 300 python bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" \
      > "$OUT/v${i}_r${rep}.json" 2>&1
    echo "$setting rep $rep: $(tail -n1 "$OUT/v${i}_r${rep}.json")"
  done
done
last=${!#}
export $last
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" > "$OUT/prof.log" 2>&1
