# Throughput sweep over batch (frames in flight) x region-growing LDS budget (diagnostic).
# Each config under its own time limit; stops at the first failure.
set -e
mkdir -p gpurun_out
for cfg in ${SWEEP:-"12288 1024" "12288 2048" "12288 3072" "8192 2048"}; do
  set -- $cfg
  echo "== LDS $1 batch $2"
  PLVI_GROW_LDS=$1 timeout -k 10 300 python bench.py --batch $2 --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err
  python -c "import json; d=json.load(open('gpurun_out/sw_$1_$2.json')); print(round(d['value']), d['ms_per_step'], d['stage_ms']['lines.region_grow'])"
done
