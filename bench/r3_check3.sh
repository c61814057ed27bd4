# blocked-pass probe + blocked GPU tests. Usage: bash bench/r3_check3.sh <tag> [probe args]
set -e
OUT=gpurun_out/${1:-r3_check3}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -k "blocked" > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench/probes/blk_probe.py "$@" > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
