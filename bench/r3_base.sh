set -e
OUT=gpurun_out/r3_base
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 ./bench/probes/gather_probe 5 > $OUT/gather_probe.jsonl 2>&1 || { cat $OUT/gather_probe.jsonl; exit 1; }
cat $OUT/gather_probe.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
