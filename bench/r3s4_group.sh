# Consumer-group Kafka (stream/group.py) on the box: GPU test, host ceiling, small bench. Usage: bash bench/r3s4_group.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s4_group}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_consumer_group.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 -u bench/probes/group_probe.py --msgs 1200000 --clients 3 > $OUT/probe.jsonl 2>&1 || { tail -20 $OUT/probe.jsonl; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 400 python3 -u bench.py --rows 200000 --rf-trees 0 --steps 5 --warmup 2 --kafka-multi-msgs 0 --kafka-msgs 200000 --kafka-confluent-msgs 100000 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print({k: (round(v) if isinstance(v, float) and v > 100 else v) for k, v in d.items() if k.startswith('kafka')})"
