#!/bin/bash
# r06: NMS candidate counters one per 128-byte line (in-tree) vs packed (variants/pad1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or stereo" > gpurun_out/r06_cpad_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_cpad_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_cpad_tests.log | head -20; exit $rc; }
for v in pad1 - pad1 -; do
  if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"; timeout -k 10 200 python -u tools/pyr_probe.py 3072 0 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
unset PLVI_LIB
CONFIGS="pad1|pad1|-;pad32|-|-" REPS=3 bash tools/ab_mix.sh
