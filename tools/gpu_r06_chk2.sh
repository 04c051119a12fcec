#!/bin/bash
# r06: checker wave after the dispatcher's compare-and-swap claim: repeatability
# (tools/mw_stress.py), the line / frame parity subset, then mw_probe timings.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
REPS=${REPS:-40} TAILN=2 bash tools/gpu_r06_stress.sh || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "lines or lsd or grow or frame or latency or stereo or orb" > gpurun_out/r06_chk_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_chk_tests.log; [ $rc -ne 0 ] && exit $rc
TESTS=0 VARIANTS="base nochk base nochk" MWB=1,64 bash tools/gpu_mw_ab.sh | cut -c1-200
