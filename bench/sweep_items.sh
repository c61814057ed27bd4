mkdir -p gpurun_out/sweep
i=0
for cfg in "8192 131072" "32768 131072" "131072 131072" "1048576 131072" "1073741824 131072" "32768 262144" "131072 65536" "8192 131072"; do
  set -- $cfg
  i=$((i+1))
  FDX_SPLIT_MIN=$1 FDX_ROW_BLOCK=$2 timeout -k 10 150 python bench/gbdt_train.py --rows 10000000 --trees 30 > gpurun_out/sweep/r$i.json 2> gpurun_out/sweep/r$i.err || exit 1
  echo "$cfg $(tail -1 gpurun_out/sweep/r$i.json)" >> gpurun_out/sweep/all.txt
done
