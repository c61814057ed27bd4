# blocked-pass probe (bench/probes/blk_probe.py). Usage: bash bench/r3_blkprobe.sh <tag> [args...]
set -e
OUT=gpurun_out/${1:-r3_blkprobe}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench/probes/blk_probe.py "$@" > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
