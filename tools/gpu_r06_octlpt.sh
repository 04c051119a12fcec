#!/bin/bash
# r06: octree grid (frames, levels) -- level 0 of every frame first (in-tree) --
# vs (levels, frames) with the level rotated by the frame (variants/octrr)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or stereo" > gpurun_out/r06_octlpt_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_octlpt_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_octlpt_tests.log | head -20; exit $rc; }
for v in octrr - octrr -; do
  if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 64,3072 0 2>&1 | grep -v amdgpu.ids | head -2 || exit 1
done
unset PLVI_LIB
CONFIGS="octrr|octrr|-;lpt|-|-" REPS=3 bash tools/ab_mix.sh
