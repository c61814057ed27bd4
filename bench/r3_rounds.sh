# per-round kernel timelines: default corpus and the wide vocabulary. Usage: bash bench/r3_rounds.sh <tag>
set -e
T=${1:-r3_rounds}
ITEMS=0 bash bench/round_probe.sh $T/narrow 8
ITEMS=0 EXTRA="--tail-words 1000000" bash bench/round_probe.sh $T/wide 8
