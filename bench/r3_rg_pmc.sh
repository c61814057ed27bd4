# Row-group pass: timing variants + PMC counters of the root pass. Usage: bash bench/r3_rg_pmc.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_rgpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/probes/rg_probe.py --slots 1,16 --wgs 1024 --alphas 4 --bins 8192 --dbg 0,2,4 > $OUT/probe.jsonl 2> $OUT/probe.err || { cat $OUT/probe.jsonl; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
CMD="bench/probes/rg_probe.py --slots 1 --wgs 1024 --alphas 4 --bins 8192 --dbg 0" OUT=$OUT/pmc MATCH=rg_hist bash bench/pmc_cmd.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr"
cat $OUT/pmc/summary.txt
