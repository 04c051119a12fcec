#!/bin/bash
# r06 (ORB chain now the longest): wave-priority variants and schedule knobs of
# the headline step, plus the multi-wave diagnostic counters with the checker.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/diagchk/libplvi_frontend.so MW_DIAG=1 timeout -k 10 200 python -u tools/mw_probe.py 1,64 \
  > gpurun_out/r06_mw_diagchk.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_mw_diagchk.txt | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
V=pl-vi-orbslam3_amd/variants
LIBS="base=;bf3=$V/bf3/libplvi_frontend.so;orb2=$V/orb2/libplvi_frontend.so;orb2bf3=$V/orb2bf3/libplvi_frontend.so" REPS=2 bash tools/ab_libs.sh || exit $?
CONFIGS="-;PLVI_GROW_SPLIT=1;PLVI_SOBEL_AFTER_GROW=0" REPS=2 bash tools/env_sweep.sh
