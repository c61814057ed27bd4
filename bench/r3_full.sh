# GPU tests + smoke, then bench/r3_bench.sh. Usage: bash bench/r3_full.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
bash bench/r3_bench.sh ${1:-r3_full}
