# RF (config 3) at 10M rows: kernel trace of a 60-tree fit, per-tree breakdown (wall vs GPU busy).
# Usage: bash bench/r3s3_rf.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s3_rf}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench/suite.py rf --trees ${TREES:-500} > $OUT/rf.json 2> $OUT/rf.err || { tail -30 $OUT/rf.err; exit 1; }
tail -1 $OUT/rf.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench/suite.py rf --trees 60 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
T=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
S=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 bench/trace_rounds.py "$T" --round 30 --marker quant_kernel --sequence > $OUT/trees.txt
head -80 $OUT/trees.txt
cp "$S" $OUT/kernel_stats.csv
rm -rf $OUT/prof
