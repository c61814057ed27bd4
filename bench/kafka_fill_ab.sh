#!/bin/bash
# Latency runs' micro-batch fill deadline (bench.py --kafka-fill-ms), 1.0 vs 0.5 ms, twice each:
# the Kafka p50 / p95 of the columnar engine, the confluent process and the consumer group.
# Usage: bash bench/kafka_fill_ab.sh <tag>
set -e
TAG=${1:-kfill}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for ms in 1.0 0.5; do
    timeout -k 10 240 python -u bench.py --rows 1000000 --rf-trees 0 --steps 10 --kafka-fill-ms $ms \
      > "$OUT/b_${ms}_$rep.json" 2> "$OUT/b_${ms}_$rep.err"
    python - "$ms" "$OUT/b_${ms}_$rep.json" <<'PY' | tee -a "$OUT/summary.jsonl"
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
keep = ("kafka_p50_ms", "kafka_p95_ms", "kafka_confluent_p50_ms", "kafka_confluent_p95_ms",
        "kafka_confluent_group_p50_ms", "kafka_confluent_group_p95_ms", "kafka_confluent_group_explain_p50_ms",
        "kafka_confluent_group_dialogues_per_s", "kafka_dialogues_per_s")
print(json.dumps({"fill_ms": float(sys.argv[1]), **{k: round(r.get(k, 0), 3) for k in keep}}))
PY
  done
done
