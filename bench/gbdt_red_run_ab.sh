#!/bin/bash
# The partial-table reduction's workgroups per thread (FDX_RG_RED_RUN): 10M-row 100-tree GBDT fit
# traced per round for each value (bench/gbdt10m_rounds.sh), rg_reduce_kernel time per round.
# (The FDX_RG_RED_RUN knob was removed after this A/B -- 32 kept, profiles/r6/gbdt_late/NOTES.md
# §8 -- so the script only re-records the default now.)
set -e
for r in "$@"; do
  FDX_RG_RED_RUN=$r bash bench/gbdt10m_rounds.sh red_run_$r 60 > /dev/null
  echo "run $r: $(grep rg_reduce_kernel gpurun_out/red_run_$r/rounds.txt | head -1)"
  tail -1 gpurun_out/red_run_$r/fit.json | grep -o '"gbdt_total_s": [0-9.]*'
done
