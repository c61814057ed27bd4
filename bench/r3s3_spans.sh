# Span breakdown of a 10M-row, 100-tree GBDT fit (quantize, row-group layout, rounds).
set -e
OUT=gpurun_out/${1:-r3s3_spans}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench/gbdt_train.py --rows 10000000 --trees 100 --trace $OUT/trace.jsonl > $OUT/run.json 2> $OUT/run.err || { tail -30 $OUT/run.err; exit 1; }
tail -1 $OUT/run.json
python3 bench/span_summary.py $OUT/trace.jsonl > $OUT/spans.txt
head -40 $OUT/spans.txt
rm -f $OUT/trace.jsonl
