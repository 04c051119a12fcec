#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=3 -k "large_batch or frame_schedule" > gpurun_out/split_tests.log 2>&1
rc=$?; tail -2 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
SWEEP="PLVI_GROW_SPLIT=1
PLVI_GROW_SPLIT=0
PLVI_GROW_SPLIT=1 PLVI_SOBEL_WITH_GROW=0" bash tools/gpu_sched_sweep.sh
