# Row-blocked histogram pass: GPU equality tests, 10M-row GBDT timing (blocked on/off), round timeline.
# Usage: bash bench/r3_blk.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_blk}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_engine.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_tree.log 2>&1 || { tail -40 $OUT/pytest_tree.log; exit 1; }
tail -2 $OUT/pytest_tree.log
for b in 1 0; do
  FDX_BLK=$b timeout -k 10 300 python -u bench/gbdt_train.py --rows 10000000 --trees 20 > $OUT/gbdt20_blk$b.json 2> $OUT/gbdt20_blk$b.err || { tail -20 $OUT/gbdt20_blk$b.err; exit 1; }
  echo "blk=$b $(cat $OUT/gbdt20_blk$b.json)"
done
ITEMS=0 bash bench/round_probe.sh ${1:-r3_blk}/probe 12 > /dev/null
head -75 $OUT/probe/rounds.txt
