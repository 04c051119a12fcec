#!/bin/bash
# A/B bench of environment settings on the GPU box:
#   tools/env_bench.sh "NAME=K1=V1,K2=V2;NAME2=..." [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
IFS=';' read -ra CFGS <<< "$1"
for c in "${CFGS[@]}"; do
  name=${c%%=*}; kv=${c#*=}
  envs=()
  [ "$kv" != "$name" ] && [ -n "$kv" ] && IFS=',' read -ra envs <<< "$kv"
  env "${envs[@]}" timeout -k 10 ${AB_T:-300} python $R/bench.py --no-cpu-baseline --no-extra --no-side ${@:2} > $R/gpurun_out/env_$name.json 2> $R/gpurun_out/env_$name.err
  rc=$?; [ $rc -ne 0 ] && { echo "$name failed rc=$rc"; tail -5 $R/gpurun_out/env_$name.err; exit $rc; }
  python - $name $R/gpurun_out/env_$name.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
s = d["stage_ms"]
print(f"{sys.argv[1]:12s} fps {d['value']:9.1f} ms/step {d['ms_per_step']:7.2f} grow {s['lines.region_grow']:7.2f} "
      f"prep {s['lines.lsd_prep']:6.2f} lbd {s['lines.lbd']:6.2f} parts {d.get('part_fps')} chk {len(d.get('oracle_check', {}).get('mismatches', []))}", flush=True)
PY
done
