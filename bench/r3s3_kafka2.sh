# Kafka config 5 (defaults: inline readers for the confluent surface only): host ceiling and the
# bench's Kafka phase on a small GBDT. Usage: bash bench/r3s3_kafka2.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s3_kafka2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 bench/probes/kafka_host_probe.py --msgs 300000 --confluent > $OUT/host_confluent.json 2>&1 || { tail -20 $OUT/host_confluent.json; exit 1; }
echo "host confluent: $(tail -1 $OUT/host_confluent.json)"
timeout -k 10 200 python3 bench/probes/kafka_timeline.py > $OUT/timeline.txt 2>&1 || { tail -20 $OUT/timeline.txt; exit 1; }
cat $OUT/timeline.txt
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --rows 200000 --rf-trees 0 --steps 5 --warmup 2 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -30 $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1])
print('bench $i', {k: (round(v) if isinstance(v, float) and v > 100 else v) for k, v in d.items() if k.startswith('kafka') and ('per_s' in k or 'ms' in k)})"
done
