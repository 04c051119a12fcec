#!/bin/bash
# r06: octree rank sort + batched node-best (in-tree) parity and bench, then
# the blur-window / Sobel-placement A/B on top of them
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_r06_octree.sh || exit $?
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/winlds/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py tests/test_frame_gpu.py -m gpu -q --timeout 240 --timeout-method thread -x > gpurun_out/r06_winlds_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_winlds_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="base|-|-;sob0|-|PLVI_SOBEL_AFTER_GROW=0;winlds|winlds|-;winlds_sob0|winlds|PLVI_SOBEL_AFTER_GROW=0;winldsbf3_sob0|winldsbf3|PLVI_SOBEL_AFTER_GROW=0" REPS=2 bash tools/ab_mix.sh
