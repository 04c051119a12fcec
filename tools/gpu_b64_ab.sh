#!/bin/bash
# batch-64 step A/B: parity subset on the first non-base variant, then
# tools/b64_probe.py per variant, REPS rounds alternating.
# usage: VARIANTS="base v1 v2" tools/gpu_b64_ab.sh   (base = the in-tree library)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
VS=${VARIANTS:-base}
for v in $VS; do
  [ $v = base ] && continue
  PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
    --timeout 120 --timeout-method thread -k "lines or frame" > gpurun_out/b64_ab_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/b64_ab_tests.log)"; [ $rc -ne 0 ] && exit $rc
  break
done
for rep in $(seq 1 ${REPS:-3}); do for v in $VS; do
  if [ $v = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  out=$(timeout -k 10 120 python -u tools/b64_probe.py 64 60 2>/dev/null | tail -1); rc=$?; echo "$v $out"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
