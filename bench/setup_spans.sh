#!/bin/bash
# Host spans of BASELINE config 2 (GBDT 1M) and config 3 (RF 10M) fits: where the fit time goes
# outside the per-level kernels (quantisation, workspace, lanes). FDX_TRACE_SYNC=1 attributes
# device time to the span that queued it. Usage: bash bench/setup_spans.sh <tag>
set -e
TAG=${1:-spans}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
FDX_TRACE=$OUT/gbdt.jsonl FDX_TRACE_SYNC=1 timeout -k 10 300 python -u bench/suite.py gbdt_1m > "$OUT/gbdt_1m.json" 2> "$OUT/gbdt_1m.err"
python bench/span_summary.py "$OUT/gbdt.jsonl" > "$OUT/gbdt_spans.txt"
python bench/span_summary.py "$OUT/gbdt.jsonl" --last > "$OUT/gbdt_spans_last.txt"
head -40 "$OUT/gbdt_spans_last.txt"
FDX_TRACE=$OUT/rf.jsonl FDX_TRACE_SYNC=1 timeout -k 10 300 python -u bench/suite.py rf > "$OUT/rf.json" 2> "$OUT/rf.err"
python bench/span_summary.py "$OUT/rf.jsonl" > "$OUT/rf_spans.txt"
python bench/span_summary.py "$OUT/rf.jsonl" --last > "$OUT/rf_spans_last.txt"
head -40 "$OUT/rf_spans_last.txt"
rm -f "$OUT/gbdt.jsonl" "$OUT/rf.jsonl"
