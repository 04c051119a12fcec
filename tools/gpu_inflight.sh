#!/bin/bash
# Batches in flight: consecutive steps alternate over
# --inflight slots; per config the FPS and ms per step.  LIBS = library
# variants (main = in-tree, others = variants/NAME), CFGS = bench arguments.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  IFS='|' read -ra CS <<< "${CFGS:---batch 3072 --inflight 1|--batch 1536 --inflight 2|--batch 3072 --inflight 2|--batch 1024 --inflight 3}"
  for cfg in "${CS[@]}"; do
    PLVI_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-side --no-check --steps 12 --warmup 3 $cfg > gpurun_out/if.json 2> gpurun_out/if.err || { echo "fail $v $cfg"; tail -3 gpurun_out/if.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/if.json'));print('$v', '$cfg', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],2))"
  done
done
