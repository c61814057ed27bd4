# blocked pass: 10M-row GBDT timing + PMC counters of the histogram kernels. Usage: bash bench/r3_blk_pmc.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_blkpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -k "blocked or device_level" > $OUT/pytest_tree.log 2>&1 || { tail -40 $OUT/pytest_tree.log; exit 1; }
tail -1 $OUT/pytest_tree.log
timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees 20 > $OUT/gbdt20.json 2> $OUT/gbdt20.err || { tail -20 $OUT/gbdt20.err; exit 1; }
cat $OUT/gbdt20.json
ROWS=10000000 TREES=2 OUT=$OUT/pmc MATCH=hist_blk bash bench/pmc_gbdt.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
cat $OUT/pmc/summary.txt
