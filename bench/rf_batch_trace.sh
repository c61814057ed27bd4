#!/bin/bash
# Kernel trace of RF 500 x depth 5 in lockstep batches on a 1.25M-row shard with forced
# collectives (the DP=8 per-rank path at world 1): GPU busy share of the forest and its kernels.
# Usage: bash bench/rf_batch_trace.sh <tag>
set -e
TAG=${1:-rfbt}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export FDX_FORCE_COLLECTIVES=1 FDX_RF_COMPACT=1
# the forest phase's wall time without the profiler (GPU events around the batch loop)
FDX_RF_EVENT_PROBE=1 timeout -k 10 300 python3 bench/suite.py rf --rows 1250000 > "$OUT/rf_events.json" 2> "$OUT/rf_events.err"
PHASE=$(python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['batch_host_s']['gpu_phase_ms'])" "$OUT/rf_events.json")
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/suite.py rf --rows 1250000 > "$OUT/rf.json" 2> "$OUT/rf.err"
tail -1 "$OUT/rf.json" | cut -c1-400
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
CP=$(find "$OUT/prof" -name "*memory_copy_trace.csv" | head -1)
python bench/trace_busy.py "$TR" --marker rf_window_threshold_lanes_kernel --top 30 --timeline 3 ${CP:+--copies "$CP"} --phase-ms "$PHASE" \
  > "$OUT/busy.txt"
cat "$OUT/busy.txt"
rm -f "$TR" "$CP"
