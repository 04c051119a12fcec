#!/bin/bash
# A/B of library variants on the headline step: LIBS = "name=path;name=path"
# ("base" = the in-tree library), REPS alternating passes of
# bench.py --no-cpu-baseline --no-extra --no-side; prints FPS, ms/step, the
# roofline kernel's in-schedule frac and the oracle check per run.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
IFS=';' read -ra LS <<< "${LIBS:-base=}"
for rep in $(seq 1 ${REPS:-2}); do
  for c in "${LS[@]}"; do
    name=${c%%=*}; path=${c#*=}
    if [ -z "$path" ]; then unset PLVI_LIB; else export PLVI_LIB=$R/$path; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-side ${BENCH_ARGS:-} > gpurun_out/ab.json 2>gpurun_out/ab.err
    rc=$?; [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -3 gpurun_out/ab.err; exit $rc; }
    echo "[$name] $(python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'))
r=d['roofline'];p=d['roofline_pyramid']
print(round(d['value']),round(d['ms_per_step'],2),'bf',round(r['avg_launch_ms'],2),round(r['frac'],3),'pyr',round(p['avg_launch_ms'],2),'mism',d['oracle_check']['mismatches'])")"
  done
done
