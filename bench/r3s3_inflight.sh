# RF trees in flight (PAR-05): GPU equality tests, then config 3 (500 trees, 10M rows) at 1/2/4/8 lanes.
# Usage: bash bench/r3s3_inflight.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s3_inflight}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tree_engine.py \
  -k "in_flight or rf" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in ${LANES:-1 2 4 8}; do
  FDX_RF_INFLIGHT=$L timeout -k 10 300 python3 bench/suite.py rf > $OUT/rf_l$L.json 2> $OUT/rf_l$L.err || { tail -30 $OUT/rf_l$L.err; exit 1; }
  echo "lanes $L: $(tail -1 $OUT/rf_l$L.json)"
done
