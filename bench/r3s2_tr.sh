# bench.py GBDT phase with span tracing + XGB-shard memory + new row-group GPU tests. Usage: bash bench/r3s2_tr.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s2_tr}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rowhist.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u bench/probes/rg_probe.py --slots 1,2,16 --wgs 1024 --alphas 16 --bins 8192 --dbg 0 --split > $OUT/probe.jsonl 2> $OUT/probe.err || { cat $OUT/probe.jsonl; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
FDX_TRACE=$OUT/trace.jsonl timeout -k 10 600 python -u bench.py --rf-trees 0 --kafka-msgs 0 --kafka-multi-msgs 0 --kafka-confluent-msgs 0 --steps 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 bench/span_summary.py $OUT/trace.jsonl > $OUT/spans.txt; head -40 $OUT/spans.txt
timeout -k 10 600 python -u bench/suite.py xgb --trees 30 > $OUT/xgb30.json 2> $OUT/xgb30.err || { tail -30 $OUT/xgb30.err; exit 1; }
cat $OUT/xgb30.json
