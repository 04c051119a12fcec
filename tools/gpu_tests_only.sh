#!/bin/bash
# GPU parity tests only (one pytest process, per-test time limit)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=12 ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|error" $OUT/gpu_tests.log | tail -25
exit $rc
