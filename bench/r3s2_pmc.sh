# PMC counters of the row-group pass, sparse part and dense part apart (root). Usage: bash bench/r3s2_pmc.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s2_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
for part in others group0; do
CMD="bench/probes/rg_probe.py --slots 1 --wgs 1024 --alphas 16 --bins 8192 --dbg 0 --only $part" OUT=$OUT/$part MATCH=rg_hist bash bench/pmc_cmd.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr"
echo "== $part"; cat $OUT/$part/summary.txt
done
