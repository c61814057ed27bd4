# CSR build test + build time, wide-vocabulary GBDT with the row-group engine. Usage: bash bench/r3s2_wide.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s2_wide}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rowhist.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench/probes/rg_probe.py --slots 1,16 --wgs 1024 --alphas 16 --bins 8192 --dbg 0 > $OUT/probe.jsonl 2> $OUT/probe.err || { cat $OUT/probe.jsonl; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
FDX_RG_MAX_GROUPS=128 timeout -k 10 600 python -u bench/gbdt_train.py --rows 10000000 --trees 20 --tail-words 1000000 > $OUT/gbdt20_wide_rg.json 2> $OUT/gbdt20_wide_rg.err || { tail -30 $OUT/gbdt20_wide_rg.err; exit 1; }
cat $OUT/gbdt20_wide_rg.json
FDX_RG_MAX_GROUPS=128 timeout -k 10 400 python -u bench/probes/rg_probe.py --tail-words 1000000 --slots 1,16 --wgs 1024,2048 --alphas 16 --bins 8192 --dbg 0 > $OUT/probe_wide.jsonl 2> $OUT/probe_wide.err || { cat $OUT/probe_wide.jsonl; tail -30 $OUT/probe_wide.err; exit 1; }
cat $OUT/probe_wide.jsonl
