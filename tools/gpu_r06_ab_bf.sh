#!/bin/bash
# r06: blur + FAST register window in LDS -- ORB / frame parity, ORB-only timing, then the step A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py tests/test_frame_gpu.py tests/test_scale_gpu.py -m gpu -q --timeout 240 --timeout-method thread -x > gpurun_out/r06_bf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06_bf_tests.log; [ $rc -eq 0 ] || exit $rc
for v in head winreg rb4 new; do
  if [ $v = new ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 3072 100000 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
unset PLVI_LIB
LIBS="head=pl-vi-orbslam3_amd/variants/head/libplvi_frontend.so;winreg=pl-vi-orbslam3_amd/variants/winreg/libplvi_frontend.so;rb4=pl-vi-orbslam3_amd/variants/rb4/libplvi_frontend.so;new=" REPS=2 bash tools/ab_libs.sh
