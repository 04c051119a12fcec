#!/bin/bash
# r06: two region-growing tasks per wave (PLVI_GROW_TPW=2: octave 0 then octave 1
# of a frame, half the resident growth waves): large-batch parity, then the step
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_GROW_TPW=2 PLVI_GROW_MW=0 timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "lines or lsd or frame or scale" > gpurun_out/r06_tpw_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_tpw_tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="base|-|-;tpw2|-|PLVI_GROW_TPW=2;tpw2_nogate|-|PLVI_GROW_TPW=2 PLVI_GROW_AFTER_BLUR=0" REPS=2 bash tools/ab_mix.sh
