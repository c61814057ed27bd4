#!/bin/bash
# RF 500 x depth 5 at 10M rows: the preselected histogram passes' active items vs launched waves
# (grower.LEVEL_STATS listed_*, from the per-level counts) and the SQ_WAVES counter summed over
# the histogram kernels' dispatches. Usage: bash bench/rf_waves_pmc.sh <tag>
set -e
TAG=${1:-rfwaves}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u bench/suite.py rf > "$OUT/rf.json" 2> "$OUT/rf.err"
python - "$OUT/rf.json" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a, w = r["listed_active_items"], r["listed_grid_waves"]
print(json.dumps({"train_only_s": r["train_only_s"], "listed_passes": r["listed_passes"], "listed_active_items": a,
                  "listed_grid_waves": w, "waves_per_active_item": round(w / max(a, 1), 3)}))
PY
PMC=/tmp/rfwaves_pmc
rm -rf "$PMC"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES --output-format csv -d "$PMC" -o run -- python3 bench/suite.py rf > /tmp/rfwaves_pmc.log 2>&1
tail -c 2000 /tmp/rfwaves_pmc.log > "$OUT/pmc_log_tail.txt"
python bench/pmc_summary.py "$PMC" --match hist_ > "$OUT/pmc_waves.txt" 2>&1 || true
head -20 "$OUT/pmc_waves.txt"
rm -rf "$PMC"
