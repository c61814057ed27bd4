# blocked-pass probe + bench/suite contract rehearsals + tree GPU tests. Usage: bash bench/r3_check2.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_check2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench/probes/blk_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 900 python -u -m pytest tests/test_bench_contract.py tests/test_tree_engine.py -m gpu -x -v --timeout 800 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -5 $OUT/pytest.log
