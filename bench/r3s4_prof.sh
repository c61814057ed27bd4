# rocprofv3 kernel stats of a full bench.py run (consumer-group phase skipped: its client processes
# would inherit the profiler's preload). Usage: bash bench/r3s4_prof.sh <tag>
set -e
OUT=gpurun_out/${1:-r3s4_prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --kafka-group-msgs 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
find $OUT/prof -type f ! -name "*stats*" -delete
find $OUT/prof -type f | head
