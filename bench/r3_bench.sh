# bench.py (N=1) + wide-vocabulary GBDT + XGB shard memory. Usage: bash bench/r3_bench.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 python -u bench/gbdt_train.py --rows 10000000 --trees 20 --tail-words 1000000 > $OUT/gbdt20_wide.json 2> $OUT/gbdt20_wide.err || { tail -30 $OUT/gbdt20_wide.err; exit 1; }
cat $OUT/gbdt20_wide.json
timeout -k 10 600 python -u bench/suite.py xgb --trees 30 > $OUT/xgb30.json 2> $OUT/xgb30.err || { tail -30 $OUT/xgb30.err; exit 1; }
cat $OUT/xgb30.json
