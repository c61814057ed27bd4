#!/bin/bash
# Row-group histogram pass with and without its flush to the level histogram (FDX_RG_DBG=4:
# timing only, trees invalid) on 1M and 10M rows: how much of rg_hist is the per-workgroup flush
# of the 8192-bin LDS tables (global integer atomics). Usage: bash bench/rg_flush_ab.sh <tag>
set -e
TAG=${1:-rgflush}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for rows in 1000000 10000000; do
  for dbg in 0 4; do
    FDX_RG_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p_${rows}_$dbg" -o run -- \
      python3 bench/gbdt_train.py --rows $rows --trees 10 > "$OUT/g_${rows}_$dbg.json" 2> "$OUT/g_${rows}_$dbg.err"
    S=$(find "$OUT/p_${rows}_$dbg" -name "*kernel_stats.csv" | head -1)
    echo "rows=$rows dbg=$dbg $(grep rg_hist_kernel "$S" | cut -d, -f1-4 | head -1)"
    find "$OUT/p_${rows}_$dbg" -name "*kernel_trace.csv" -delete
  done
done
