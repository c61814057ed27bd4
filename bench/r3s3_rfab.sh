# RF config 3 A/B: sampled-pass settings (env pairs) at 4 lanes, two runs each.
set -e
OUT=gpurun_out/${1:-r3s3_rfab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_engine.py \
  -k "sampled or in_flight or rf" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for CFG in "FDX_RF_SAMPLED=1" "FDX_RF_SAMPLED=0" "FDX_RF_SAMPLED=1 FDX_RF_LISTED_NODES=0" "FDX_RF_SAMPLED=1" "FDX_RF_SAMPLED=0"; do
  i=$((i+1))
  env $CFG timeout -k 10 300 python3 bench/suite.py rf > $OUT/rf_$i.json 2> $OUT/rf_$i.err || { tail -30 $OUT/rf_$i.err; exit 1; }
  echo "$CFG: $(python3 -c "import json;d=json.loads(open('$OUT/rf_$i.json').read().splitlines()[-1]);print(round(d['train_only_s'],3), d['accuracy'])")"
done
