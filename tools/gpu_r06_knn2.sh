#!/bin/bash
# r06: the step's ORB kNN-2 behind the line chain (PLVI_KNN_ON_CRIT=1) now that
# the ORB chain is the busier one: frame parity with it, then the headline A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_KNN_ON_CRIT=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "frame or scale or c4" > gpurun_out/r06_knn2_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_knn2_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_knn2_tests.log | head; exit $rc; }
CONFIGS="base|-|-;knn|-|PLVI_KNN_ON_CRIT=1" REPS=3 bash tools/ab_mix.sh
