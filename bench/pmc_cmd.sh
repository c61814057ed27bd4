#!/bin/bash
# PMC counter passes over any python command on one MI355X: one rocprofv3 run per argument, each
# argument a space-separated counter group within the per-block hardware limits (<= 8 SQ,
# 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM). Usage (GPU box, repo root):
#   CMD="bench/probes/rg_probe.py --slots 1" OUT=gpurun_out/pmc MATCH=rg_hist bash bench/pmc_cmd.sh "SQ_WAVES SQ_INSTS_LDS" ...
set -e
OUT=${OUT:-gpurun_out/pmc_cmd}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
dirs=()
for group in "$@"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $group --output-format csv -d "$OUT/p$i" -o run -- \
    python3 $CMD > "$OUT/p$i.log" 2>&1
  dirs+=("$OUT/p$i")
done
python3 bench/pmc_summary.py "${dirs[@]}" --match "${MATCH:-fdx::}" > "$OUT/summary.txt"
if [ -z "$KEEP_RAW" ]; then rm -rf "${dirs[@]}"; fi
