#!/bin/bash
# r06: candidate lists + octree over partitioned per-node ranges (in-tree lib),
# the describe pipeline on top of it, and the HEAD library: ORB parity subset, then A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or scale or stereo or c4 or vocab or bow" > gpurun_out/r06_part_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_part_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_part_tests.log | head -20; exit $rc; }
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/descpipe/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame" > gpurun_out/r06_descpipe_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_descpipe_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_descpipe_tests.log | head; exit $rc; }
for v in head - descpipe; do
  if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 64,3072 0 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
done
unset PLVI_LIB
CONFIGS="head|head|-;part|-|-;descpipe|descpipe|-" REPS=3 bash tools/ab_mix.sh
