#!/bin/bash
# r06: blur + FAST with its 7-row window in LDS (64 VGPRs: two waves beside six
# growth waves), ORB parity on the variant, then the step A/B with and without
# the Sobel pyramid beside growth (PLVI_SOBEL_AFTER_GROW=0), and ORB-only timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/winlds/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py tests/test_frame_gpu.py tests/test_scale_gpu.py -m gpu -q --timeout 240 --timeout-method thread -x > gpurun_out/r06_winlds_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_winlds_tests.log; [ $rc -eq 0 ] || exit $rc
for v in - winlds; do
  if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 3072 0 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
unset PLVI_LIB
CONFIGS="base|-|-;sob0|-|PLVI_SOBEL_AFTER_GROW=0;winlds|winlds|-;winlds_sob0|winlds|PLVI_SOBEL_AFTER_GROW=0;winldsbf3_sob0|winldsbf3|PLVI_SOBEL_AFTER_GROW=0" REPS=2 bash tools/ab_mix.sh
