#!/bin/bash
# r06: multi-wave repeatability, in-tree (checker) and nochk libraries
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for v in base nochk; do
  if [ $v = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/mw_stress.py 16 ${REPS:-30} > gpurun_out/r06_stress_$v.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r06_stress_$v.txt | tail -${TAILN:-6}; [ $rc -ne 0 ] && exit $rc
done
exit 0
