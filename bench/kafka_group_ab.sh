#!/bin/bash
# Consumer-group placement A/B: the box's CPU topology, the instant-scorer host
# ceiling (bench/probes/group_probe.py) and bench.py's Kafka phases under each client placement:
#   nopin  FDX_GROUP_PIN=0                  clients float over the scorer's CPUs (its NUMA node)
#   coreN  N whole cores per client (SMT siblings included)
#   poolN  the clients share 3N whole cores, the scorer keeps the rest
# (first A/B, profiles/r6/kafka/group_ab1.jsonl: 2 logical CPUs per client 1.14 M/s, 2 cores 1.24,
#  3 cores 1.39, unpinned 1.51)
# Usage: bash bench/kafka_group_ab.sh <tag>
set -e
TAG=${1:-kab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
{
  echo "nproc=$(nproc) affinity=$(python -c 'import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:4], a[-4:])')"
  for c in 0 1 58 63 128 186 191; do
    f=/sys/devices/system/cpu/cpu$c/topology/thread_siblings_list
    [ -r $f ] && echo "cpu$c siblings $(cat $f)"
  done
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
} > "$OUT/topology.txt"
cat "$OUT/topology.txt"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --rows 1000000 --rf-trees 0 --steps 10 \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  python - "$name" "$OUT/bench_$name.json" <<'EOF' | tee -a "$OUT/summary.jsonl"
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
keep = ("kafka_confluent_group_dialogues_per_s", "kafka_confluent_group_p50_ms", "kafka_confluent_group_p95_ms",
        "kafka_confluent_group_client_dialogues_per_s", "kafka_confluent_group_client_cpu_util",
        "kafka_confluent_group_client_cpus", "kafka_confluent_group_client_numa", "kafka_confluent_group_pinned",
        "kafka_confluent_dialogues_per_s", "kafka_confluent_p50_ms", "kafka_dialogues_per_s",
        "kafka_multi_gpu_dialogues_per_s", "kafka_confluent_group_runs_dialogues_per_s",
        "kafka_confluent_group_host_busy_cpus", "kafka_confluent_group_cgroup_busy_cpus",
        "kafka_confluent_group_cgroup_quota_cpus", "kafka_confluent_group_throttled_ms")
print(json.dumps({"variant": sys.argv[1], **{k: r.get(k) for k in keep}}))
EOF
}
for rep in 1 2 3; do
  run nopin_$rep FDX_GROUP_PIN=0
  run pool4_$rep FDX_GROUP_SHARED=1 FDX_GROUP_CPUS_PER_CLIENT=4
  run pool8_$rep FDX_GROUP_SHARED=1 FDX_GROUP_CPUS_PER_CLIENT=8
done
