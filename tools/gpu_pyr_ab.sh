#!/bin/bash
# pyramid frames-per-workgroup A/B: ORB parity with each variant, then the bench sweep
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for v in pyr2 pyr1; do
  PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --maxfail=3 -k "orb" > gpurun_out/pa_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/pa_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
SWEEP="X=1
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/pyr2/libplvi_frontend.so
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/pyr1/libplvi_frontend.so" bash tools/gpu_sched_sweep.sh
