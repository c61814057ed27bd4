# Row-group + stream GPU tests, build timing, full bench. Usage: bash bench/r3s2_k.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s2_k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rowhist.py tests/test_stream_engine.py tests/test_serving.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
FDX_RG_TIMING=1 timeout -k 10 300 python -u bench/probes/rg_probe.py --slots 1 --wgs 1024 --alphas 16 --bins 8192,8192 --dbg 0 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
