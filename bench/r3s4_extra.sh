# RF alone, featurize probe, XGB 1000 trees on one 12.5M-row shard, RCCL two-ranks-one-GPU probe. Usage: bash bench/r3s4_extra.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s4_extra}
mkdir -p $OUT
export TMPDIR=/tmp
nproc; cat /proc/loadavg
timeout -k 10 300 python3 -u bench/suite.py rf > $OUT/rf.json 2> $OUT/rf.err || { tail -30 $OUT/rf.err; exit 1; }
cat $OUT/rf.json
FDX_RF_INFLIGHT=1 timeout -k 10 300 python3 -u bench/suite.py rf > $OUT/rf_inflight1.json 2> $OUT/rf1.err || { tail -30 $OUT/rf1.err; exit 1; }
cat $OUT/rf_inflight1.json
timeout -k 10 300 python3 -u bench/probes/feat_probe.py > $OUT/feat_probe.jsonl 2>&1 || { tail -30 $OUT/feat_probe.jsonl; exit 1; }
cat $OUT/feat_probe.jsonl
timeout -k 10 400 python3 -u bench/suite.py xgb --trees 1000 > $OUT/xgb1000.json 2> $OUT/xgb1000.err || { tail -30 $OUT/xgb1000.err; exit 1; }
cat $OUT/xgb1000.json
timeout -k 10 90 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench/probes/rccl_same_gpu.py > $OUT/rccl.log 2>&1 && echo "rccl same-gpu: OK" || echo "rccl same-gpu: FAILED"
tail -5 $OUT/rccl.log
