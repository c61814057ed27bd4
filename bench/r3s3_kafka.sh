# Kafka config 5 through the confluent surface: host ceiling (instant scorer) and the bench's Kafka
# phase on a small GBDT (100 trees), reader threads vs inline readers. Usage: bash bench/r3s3_kafka.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s3_kafka}
mkdir -p $OUT
export TMPDIR=/tmp
for M in 0 1; do
  FDX_STREAM_INLINE=$M timeout -k 10 200 python3 bench/probes/kafka_host_probe.py --msgs 300000 --confluent > $OUT/host_i$M.json 2>&1 || { tail -20 $OUT/host_i$M.json; exit 1; }
  echo "host inline=$M: $(tail -1 $OUT/host_i$M.json)"
done
timeout -k 10 200 python3 bench/probes/kafka_host_probe.py --msgs 1000000 > $OUT/host_columnar.json 2>&1 || { tail -20 $OUT/host_columnar.json; exit 1; }
echo "host columnar: $(tail -1 $OUT/host_columnar.json)"
for M in 0 1; do
  FDX_STREAM_INLINE=$M timeout -k 10 400 python3 bench.py --rows 200000 --rf-trees 0 --steps 5 --warmup 2 > $OUT/bench_i$M.json 2> $OUT/bench_i$M.err || { tail -30 $OUT/bench_i$M.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_i$M.json').read().strip().splitlines()[-1])
print('bench inline=$M', {k: (round(v) if isinstance(v, float) and v > 100 else v) for k, v in d.items() if k.startswith('kafka')})"
done
