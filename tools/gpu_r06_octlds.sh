#!/bin/bash
# r06: octree LDS stage size (PLVI_ORB_OCT_LDS: candidates staged per wave;
# smaller = more octree waves per CU, more levels on the memory-scan path):
# ORB parity subset, ORB-only chain at 3072 frames per setting, headline A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or stereo" > gpurun_out/r06_octlds_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_octlds_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_octlds_tests.log | head -20; exit $rc; }
for v in 1536 1024 768 512 256; do
  echo "== PLVI_ORB_OCT_LDS=$v"; PLVI_ORB_OCT_LDS=$v timeout -k 10 200 python -u tools/pyr_probe.py 3072 0 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
CONFIGS="l1536|-|PLVI_ORB_OCT_LDS=1536;l1024|-|PLVI_ORB_OCT_LDS=1024;l768|-|PLVI_ORB_OCT_LDS=768" REPS=2 bash tools/ab_mix.sh
