#!/bin/bash
# r06: commit-driven revalidation (checker wave) A/B: parity subset on the
# in-tree library (checker on), the diagnostic counters with and without the
# checker, then mw_probe timings (nochk = r05 scheme) alternated.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "lines or lsd or grow or frame or latency" > gpurun_out/r06_chk_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r06_chk_tests.log; [ $rc -ne 0 ] && exit $rc; fi
for v in diagchk diag; do
  PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so MW_DIAG=1 timeout -k 10 200 python -u tools/mw_probe.py 1,64 \
    > gpurun_out/r06_mw_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -v amdgpu.ids gpurun_out/r06_mw_$v.txt | cut -c1-900; [ $rc -ne 0 ] && exit $rc
done
TESTS=0 VARIANTS="base nochk base nochk" MWB=1,64 bash tools/gpu_mw_ab.sh
