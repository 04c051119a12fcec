#!/bin/bash
# NMS register-streaming A/B: ORB parity (main + single-buffer variant), bench sweep vs HEAD (variants/base)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for L in "" $R/pl-vi-orbslam3_amd/variants/nmssb/libplvi_frontend.so; do
  PLVI_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --maxfail=3 -k "orb or frame" > gpurun_out/nms_tests.log 2>&1
  rc=$?; echo "[$L] $(tail -1 gpurun_out/nms_tests.log)"; [ $rc -ne 0 ] && exit $rc
done
SWEEP="PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/base/libplvi_frontend.so
X=1
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/nmssb/libplvi_frontend.so
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/base/libplvi_frontend.so
X=1" bash tools/gpu_sched_sweep.sh
