#!/bin/bash
# Plain-timing sweep of GBDT knobs (10M rows, 20 trees); one JSON line per setting.
# Usage (GPU box, repo root): bash bench/sweep_gbdt.sh <outfile> "ENV=a" "ENV=b" ...
set -e
OUT=$1; shift
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for SETTING in "$@"; do
  R=$(env $SETTING timeout -k 10 200 python bench/gbdt_train.py --rows 10000000 --trees 20 2>/dev/null | tail -1)
  echo "{\"setting\": \"$SETTING\", \"result\": $R}" | tee -a "$OUT"
done
