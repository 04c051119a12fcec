#!/bin/bash
# r06: two-stage describe pipeline (PLVI_DESC_PIPE=1: next keypoint's blur box by
# global_load_lds) re-measured under one growth task per wave, where the
# describe runs beside six growth waves per SIMD (2 describe waves per SIMD)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/descpipe/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or stereo" > gpurun_out/r06_descpipe2_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_descpipe2_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_descpipe2_tests.log | head; exit $rc; }
CONFIGS="base|-|-;descpipe|descpipe|-" REPS=3 bash tools/ab_mix.sh
