# GPU tests + gather probe + bench (round 3 checks). Usage: bash bench/r3_check.sh <tag>
set -e
OUT=gpurun_out/${1:-r3_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 ./bench/probes/gather_probe 5 > $OUT/gather_probe.jsonl 2>&1 || { cat $OUT/gather_probe.jsonl; exit 1; }
grep -E '"g8s1_xcd"|"g16_xcd"|"g8_xcd"' $OUT/gather_probe.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
