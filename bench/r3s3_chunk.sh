# RF sampled passes vs item size (FDX_HIST_CHUNK): probe + config-3 bench per chunk, pack/list on and off.
set -e
OUT=gpurun_out/${1:-r3s3_chunk}
mkdir -p $OUT
export TMPDIR=/tmp
for CH in ${CHUNKS:-32768 8192 2048}; do
  FDX_HIST_CHUNK=$CH timeout -k 10 300 python3 bench/probes/rf_probe.py --trees 0 > $OUT/probe_c$CH.jsonl 2> $OUT/probe_c$CH.err || { tail -20 $OUT/probe_c$CH.err; exit 1; }
  echo "chunk $CH"; cut -c1-60,330-520 $OUT/probe_c$CH.jsonl
  for S in 1 0; do
    FDX_HIST_CHUNK=$CH FDX_RF_SAMPLED=$S timeout -k 10 300 python3 bench/suite.py rf > $OUT/rf_c${CH}_s$S.json 2> $OUT/rf_c${CH}_s$S.err || { tail -30 $OUT/rf_c${CH}_s$S.err; exit 1; }
    echo "chunk $CH sampled $S: $(tail -1 $OUT/rf_c${CH}_s$S.json | cut -c1-260)"
  done
done
