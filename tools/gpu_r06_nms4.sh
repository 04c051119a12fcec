#!/bin/bash
# r06: NMS with 4 rows per round trip (33 VGPRs: 3 waves beside six growth
# waves per SIMD instead of 2 at 41) vs 8 (in-tree)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/nms4/libplvi_frontend.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame" > gpurun_out/r06_nms4_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_nms4_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_nms4_tests.log | head -20; exit $rc; }
for v in nms4 - ; do
  if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 64,3072 0 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
done
unset PLVI_LIB
CONFIGS="rows8|-|-;nms4|nms4|-" REPS=3 bash tools/ab_mix.sh
