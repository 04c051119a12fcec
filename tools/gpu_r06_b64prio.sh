#!/bin/bash
# r06: batch-64 leg vs the ORB stream priority of the large-batch handles
# (default: least for >= 1024-frame handles; PLVI_ORB_PRIO=1: greatest for all)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in ${B64_REPS:-1 2}; do
  for c in ${B64_CONFIGS:-"-" "PLVI_ORB_PRIO=1"}; do
    e=$c; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b64p.json 2> gpurun_out/b64p.err || { tail -3 gpurun_out/b64p.err; exit 1; }
    echo "[$c] $(python3 -c "
import json;d=json.load(open('gpurun_out/b64p.json'));r=d['roofline']
print(round(d['value']), round(d['ms_per_step'],2), 'frac', round(r['frac'],3), 'b64', round(d['batch64']['value']), round(d['batch64']['ms_per_step'],3), 'lat', round(d['single_frame_latency']['drop_in_process']['median_ms'],2))")"
  done
done
