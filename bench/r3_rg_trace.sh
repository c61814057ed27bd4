# Row-group engine: kernel trace of a 10M-row GBDT run, per-round breakdown. Usage: bash bench/r3_rg_trace.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_rgtrace}
mkdir -p $OUT
export TMPDIR=/tmp
FDX_ROWHIST=${FDX_ROWHIST:-1} timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench/gbdt_train.py --rows 10000000 --trees 12 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
T=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
S=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 bench/trace_rounds.py "$T" --round 6 > $OUT/rounds.txt
head -40 $OUT/rounds.txt
cp "$S" $OUT/kernel_stats.csv
rm -rf $OUT/prof
