#!/bin/bash
# PMC counter passes over a short GBDT run on one MI355X (one rocprofv3 run per counter group,
# each within the per-block hardware limits). Usage (GPU box, repo root):
#   bash bench/pmc_gbdt.sh [rows] [trees] [outdir]
set -e
ROWS=${1:-2000000}
TREES=${2:-3}
OUT=${3:-gpurun_out/pmc_gbdt}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1
  shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$tag" -o run -- \
    python3 bench/gbdt_train.py --rows "$ROWS" --trees "$TREES" > "$OUT/$tag.log" 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_ANY TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE
run mem TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
