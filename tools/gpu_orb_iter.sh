#!/bin/bash
# ORB iteration: parity tests for ORB + pyramid-kernel timing (rocprof stats of tools/orb_micro.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ "${PYTEST_K:-x}" != none ]; then timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=3 -k "${PYTEST_K:-orb or compat or scale}" > $OUT/gpu_tests_q.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests_q.log; [ $rc -ne 0 ] && exit $rc; fi
bash tools/ab_kernel.sh "${VARIANTS:-main}" "${KERNEL:-orb_pyramid}" 3072 5
