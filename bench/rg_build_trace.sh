#!/bin/bash
# Kernel durations of the row-group layout build (models/quantize.RowGroups, csrc/row_kernels.hip
# rg_build_csr_count / _place and the scan) at ROWS rows. Usage: ROWS=10000000 bash bench/rg_build_trace.sh <tag>
set -e
TAG=${1:-rgb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/probes/rg_build_timing.py > "$OUT/rg.txt" 2>&1
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 - "$TR" > "$OUT/build_kernels.txt" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rg_build" in r["Kernel_Name"] or "dense_scatter" in r["Kernel_Name"]]
for r in rows[-8:]:
    print(f'{(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:10.1f} us  {r["Kernel_Name"][:90]}')
PY
cat "$OUT/build_kernels.txt"
rm -f "$TR"
