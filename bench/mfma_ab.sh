#!/bin/bash
# MFMA vs LDS-atomic histogram engines, measured. GBDT 10M rows x 20 trees:
# FDX_ROWHIST=0 (i8-MFMA CSC passes + dense MFMA path) vs 1 (row-group LDS-atomic engine, default);
# RF 500 trees: FDX_RF_LDS=0 (i8 MFMA) vs 1 (LDS atomics, default); then PMC of the MFMA kernels
# (MFMA busy cycles, VALU / LDS instructions) and of rg_hist. Usage: bash bench/mfma_ab.sh <tag>
set -e
TAG=${1:-mfma}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for RH in 1 0; do
  FDX_ROWHIST=$RH timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees 20 > "$OUT/gbdt_rowhist$RH.json" 2> "$OUT/gbdt_rowhist$RH.err"
  echo "rowhist $RH $(tail -1 $OUT/gbdt_rowhist$RH.json)"
done
FDX_ROWHIST=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rh0" -o run -- \
  python3 bench/gbdt_train.py --rows 10000000 --trees 20 > "$OUT/prof_rh0.log" 2>&1
find "$OUT/prof_rh0" -name "*kernel_trace.csv" -delete
head -14 $(find "$OUT/prof_rh0" -name "*kernel_stats.csv") | cut -c1-200
for LDS in 1 0; do
  FDX_RF_LDS=$LDS timeout -k 10 300 python -u bench/suite.py rf > "$OUT/rf_lds$LDS.json" 2> "$OUT/rf_lds$LDS.err"
  echo "rf lds $LDS $(tail -1 $OUT/rf_lds$LDS.json | cut -c1-300)"
done
export FDX_ROWHIST=0
CMD="bench/gbdt_train.py --rows 10000000 --trees 2" OUT=$OUT/pmc_mfma MATCH="fdx::" bash bench/pmc_cmd.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  || echo "pmc pass failed"
cat "$OUT/pmc_mfma/summary.txt" | head -40
