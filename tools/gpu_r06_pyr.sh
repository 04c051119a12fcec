#!/bin/bash
# r06: pyramid builders -- ORB parity tests, then tools/pyr_probe.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py tests/test_libm.py -m gpu -v --timeout 240 --timeout-method thread -x > gpurun_out/r06_orb_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r06_orb_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pyr_probe.py ${PROBE_B:-1,8,64,256,512,1024,3072} ${PROBE_MODES:-0,100000} > gpurun_out/r06_pyr_probe.txt 2>&1
rc=$?; cat gpurun_out/r06_pyr_probe.txt; exit $rc
