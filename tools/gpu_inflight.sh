set -u
mkdir -p gpurun_out
for cfg in "--batch 3072 --inflight 1" "--batch 3072 --inflight 2" "--batch 1536 --inflight 2" "--batch 1536 --inflight 3"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-side --no-check --steps 12 --warmup 3 $cfg > gpurun_out/if.json 2> gpurun_out/if.err || { echo "fail $cfg"; tail -3 gpurun_out/if.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/if.json'));print('$cfg', round(d['value']), round(d['ms_per_step'],2))"
done
