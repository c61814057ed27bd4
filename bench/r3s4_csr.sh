set -e
OUT=gpurun_out/${1:-r3s4_csr}
mkdir -p $OUT
export TMPDIR=/tmp
cat /proc/loadavg
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 -u bench/probes/feat_probe.py --cold > $OUT/cold.jsonl 2>&1 || { tail -30 $OUT/cold.jsonl; exit 1; }
cat $OUT/cold.jsonl
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
