# Row-group engine: GPU tests, probe (timing + bitwise equality vs the CSC passes), GBDT run.
# Usage: bash bench/r3_rg.sh <tag> [probe args]
set -e
OUT=gpurun_out/${1:-r3_rg}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rowhist.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u bench/probes/rg_probe.py "$@" > $OUT/probe.jsonl 2> $OUT/probe.err || { cat $OUT/probe.jsonl; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
FDX_ROWHIST=1 timeout -k 10 400 python -u bench/gbdt_train.py --rows 10000000 --trees 20 > $OUT/gbdt20_rg.json 2> $OUT/gbdt20_rg.err || { tail -30 $OUT/gbdt20_rg.err; exit 1; }
cat $OUT/gbdt20_rg.json
