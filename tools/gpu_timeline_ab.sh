#!/bin/bash
# Step timelines of library variants (rocprofv3 kernel trace of a short bench
# run each): LIBS="main nmsfill" ARGS="--inflight 1" bash tools/gpu_timeline_ab.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  cd /tmp && export TMPDIR=/tmp
  PLVI_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tl_$v -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-check --no-extra --no-side --steps 4 --warmup 2 ${ARGS:-} > $OUT/tl_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $OUT/tl_$v.log; exit 1; }
  cd $R
  T=$(find $OUT/tl_$v -name "run_kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $T > $OUT/step_timeline_$v.txt; echo "== $v"; cat $OUT/step_timeline_$v.txt
  find $OUT/tl_$v -name "*.csv" -size +20M -delete
done
