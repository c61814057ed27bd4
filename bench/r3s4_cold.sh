set -e
OUT=gpurun_out/${1:-r3s4_cold}
mkdir -p $OUT
export TMPDIR=/tmp
cat /proc/loadavg
timeout -k 10 300 python3 -u bench/probes/feat_probe.py --cold > $OUT/cold.jsonl 2>&1 || { tail -30 $OUT/cold.jsonl; exit 1; }
cat $OUT/cold.jsonl
