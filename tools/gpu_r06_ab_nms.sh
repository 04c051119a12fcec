#!/bin/bash
# r06: NMS / SAT rows-in-flight A/B (ORB parity subset on the combined variant,
# then the headline step per variant), plus the multi-wave diagnostic probe.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/ns/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
  --timeout 120 --timeout-method thread -k "orb or frame or scale" > gpurun_out/r06_ns_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_ns_tests.log; [ $rc -ne 0 ] && exit $rc
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/diag/libplvi_frontend.so MW_DIAG=1 timeout -k 10 200 python -u tools/mw_probe.py 1,64 \
  > gpurun_out/r06_mw_diag.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_mw_diag.txt; [ $rc -ne 0 ] && exit $rc
LIBS="base=;nms40=pl-vi-orbslam3_amd/variants/nms40/libplvi_frontend.so;sat32=pl-vi-orbslam3_amd/variants/sat32/libplvi_frontend.so;ns=pl-vi-orbslam3_amd/variants/ns/libplvi_frontend.so" REPS=2 bash tools/ab_libs.sh
