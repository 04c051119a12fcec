#!/bin/bash
# Schedule sweep: bench FPS per line of SWEEP, each 'ENV=V ... -- --bench-args'.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
i=0
while IFS= read -r cfg; do
  [ -z "$cfg" ] && continue
  i=$((i+1))
  envs=${cfg%%--*}; args=""; [[ "$cfg" == *--* ]] && args=${cfg#*--}
  env X_=1 $envs timeout -k 10 300 python bench.py --steps 10 --no-extra --no-side --no-cpu-baseline --no-check $args > $OUT/sw_$i.json 2> $OUT/sw_$i.err
  rc=$?; [ $rc -ne 0 ] && { echo "[$cfg] rc=$rc"; tail -3 $OUT/sw_$i.err; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/sw_$i.json')); print('[$cfg]', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'blur_ms', round(d['roofline']['avg_launch_ms'],2))"
done <<< "${SWEEP}"
