#!/bin/bash
# r06: the step's ORB kNN-2 on the line stream (PLVI_KNN_ON_CRIT) and two growth
# tasks per wave (PLVI_GROW_TPW=2), alone and together
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_KNN_ON_CRIT=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "frame or scale or c4" > gpurun_out/r06_knn_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_knn_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="base|-|-;knn|-|PLVI_KNN_ON_CRIT=1;tpw2|-|PLVI_GROW_TPW=2;tpw2knn|-|PLVI_GROW_TPW=2 PLVI_KNN_ON_CRIT=1" REPS=3 bash tools/ab_mix.sh
