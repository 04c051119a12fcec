#!/bin/bash
# A/B bench of library variants on the GPU box: tools/ab_bench.sh "main prio ..." [bench args]
# "main" = lib/libplvi_frontend.so, other names = variants/NAME (tools/build_variant.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for v in $1; do
  if [ "$v" = main ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  PLVI_LIB=$L timeout -k 10 ${AB_T:-300} python $R/bench.py --no-cpu-baseline --no-side --no-extra --no-check \
    --steps 10 --warmup 2 ${@:2} > $R/gpurun_out/ab_$v.json 2> $R/gpurun_out/ab_$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "$v failed rc=$rc"; tail -5 $R/gpurun_out/ab_$v.err; exit $rc; }
  python - $v $R/gpurun_out/ab_$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
s = d["stage_ms"]
print(f"{sys.argv[1]:10s} fps {d['value']:9.1f} ms/step {d['ms_per_step']:7.2f} bf_ms {d['roofline']['avg_launch_ms']:6.2f} "
      f"grow {s['lines.region_grow']:7.2f} nms {s['orb.nms']:6.2f} parts {d.get('part_fps')}")
PY
done
# env A/B: AB_ENVS="name:VAR=v,VAR2=v ..." runs the in-tree library under each environment
for spec in ${AB_ENVS:-}; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 ${AB_T:-300} python $R/bench.py --no-cpu-baseline --no-side --no-extra --no-check \
    --steps 10 --warmup 2 > $R/gpurun_out/ab_$name.json 2> $R/gpurun_out/ab_$name.err
  rc=$?; [ $rc -ne 0 ] && { echo "$name failed rc=$rc"; tail -5 $R/gpurun_out/ab_$name.err; exit $rc; }
  python - $name $R/gpurun_out/ab_$name.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
s = d["stage_ms"]
print(f"{sys.argv[1]:10s} fps {d['value']:9.1f} ms/step {d['ms_per_step']:7.2f} bf_ms {d['roofline']['avg_launch_ms']:6.2f} "
      f"grow {s['lines.region_grow']:7.2f} nms {s['orb.nms']:6.2f} parts {d.get('part_fps')}")
PY
done
