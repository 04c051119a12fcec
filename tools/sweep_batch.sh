# Throughput sweep over region-growing LDS budget x batch (diagnostic).
set -e
for cfg in ${SWEEP:-"12288 1024" "12288 512" "20480 512" "8192 2048"}; do
  set -- $cfg
  PLVI_GROW_LDS=$1 timeout -k 10 300 python bench.py --batch $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err
done
