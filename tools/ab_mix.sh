#!/bin/bash
# A/B of (library variant, schedule environment) pairs on the headline step:
# CONFIGS = "name|variant|ENV=V ENV2=V;..." (variant "-" = the in-tree library,
# env "-" = none), REPS alternating passes of bench.py --no-cpu-baseline
# --no-extra --no-side; prints FPS, ms/step, the roofline kernel's timed launch
# and frac, the pyramid's, and the oracle check.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
IFS=';' read -ra CS <<< "${CONFIGS:?}"
for rep in $(seq 1 ${REPS:-2}); do
  for c in "${CS[@]}"; do
    IFS='|' read -r name var envs <<< "$c"
    if [ "$var" = "-" ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$var/libplvi_frontend.so; fi
    [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-side ${BENCH_ARGS:-} > gpurun_out/ab.json 2>gpurun_out/ab.err
    rc=$?; [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -3 gpurun_out/ab.err; exit $rc; }
    echo "[$name] $(python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'))
r=d['roofline'];p=d['roofline_pyramid']
print(round(d['value']),round(d['ms_per_step'],2),'bf',round(r['avg_launch_ms'],2),round(r['frac'],3),'pyr',round(p['avg_launch_ms'],2),'mism',d['oracle_check']['mismatches'])")"
  done
done
