#!/bin/bash
# schedule-knob sweep of the headline step: each line of $CONFIGS is an env
# assignment list ("-" = defaults), REPS bench runs each, alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
IFS=';' read -ra CS <<< "${CONFIGS:--}"
for rep in $(seq 1 ${REPS:-2}); do
  for c in "${CS[@]}"; do
    if [ "$c" = "-" ]; then envs=""; else envs="$c"; fi
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-side ${BENCH_ARGS:-} > gpurun_out/es.json 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; exit $rc; }
    echo "[$c] $(python3 -c "import json;d=json.load(open('gpurun_out/es.json'));print(round(d['value']),round(d['ms_per_step'],2),d['oracle_check']['mismatches'])")"
  done
done
