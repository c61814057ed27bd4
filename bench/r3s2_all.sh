# Session check: row-group probe, GBDT trace, all GPU tests + smoke, bench.py, wide-vocab GBDT, XGB shard.
# Usage: bash bench/r3s2_all.sh <tag>
set -e
T=${1:-r3s2_all}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench/probes/rg_probe.py --slots 1,2,16 --wgs 1024 --alphas 16 --bins 8192 --dbg 0 --split > $OUT/probe.jsonl 2> $OUT/probe.err || { cat $OUT/probe.jsonl; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
bash bench/r3_rg_trace.sh $T/trace
bash bench/r3_full.sh $T
