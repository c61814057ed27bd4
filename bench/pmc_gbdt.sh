#!/bin/bash
# PMC counter passes over a short GBDT run on one MI355X: one rocprofv3 run per argument, each
# argument a space-separated counter group within the per-block hardware limits (<= 8 SQ,
# 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM). Usage (GPU box, repo root):
#   ROWS=2000000 TREES=3 OUT=gpurun_out/pmc bash bench/pmc_gbdt.sh "SQ_WAVES SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum"
set -e
ROWS=${ROWS:-2000000}
TREES=${TREES:-3}
OUT=${OUT:-gpurun_out/pmc_gbdt}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
dirs=()
for group in "$@"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench/gbdt_train.py --no-warmup --rows "$ROWS" --trees "$TREES" ${RG_DBG:+--rg-dbg $RG_DBG} > "$OUT/p$i.log" 2>&1
  dirs+=("$OUT/p$i")
done
# the raw per-dispatch CSVs of a 10M-row run exceed what gpurun copies back: keep the summary
python3 bench/pmc_summary.py "${dirs[@]}" --match "${MATCH:-fdx::}" > "$OUT/summary.txt"
if [ -z "$KEEP_RAW" ]; then rm -rf "${dirs[@]}"; fi
