set -e
OUT=gpurun_out/${1:-r3s4_contract}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_contract.py tests/test_consumer_group.py -m gpu -x -v --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
