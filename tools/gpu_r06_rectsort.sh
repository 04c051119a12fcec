#!/bin/bash
# r06: large-batch region2rect over size-sorted regions (PLVI_RECT_SORTED):
# line / frame parity subset, then the headline A/B (sorted default vs off)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "line or lsd or frame or rect" > gpurun_out/r06_rectsort_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_rectsort_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_rectsort_tests.log | head -20; exit $rc; }
CONFIGS="sorted|-|-;unsorted|-|PLVI_RECT_SORTED=0" REPS=3 bash tools/ab_mix.sh
