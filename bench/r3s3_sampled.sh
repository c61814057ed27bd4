# RF sampled passes (packed row state + listed items): GPU tests, probe, config-3 bench.
# Usage: bash bench/r3s3_sampled.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s3_sampled}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tree_engine.py \
  -k "sampled or in_flight or rf" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 bench/probes/rf_probe.py --trees 0,1 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
for S in 1 0; do
  FDX_RF_SAMPLED=$S timeout -k 10 300 python3 bench/suite.py rf > $OUT/rf_s$S.json 2> $OUT/rf_s$S.err || { tail -30 $OUT/rf_s$S.err; exit 1; }
  echo "sampled $S: $(tail -1 $OUT/rf_s$S.json)"
done
