#!/bin/bash
# drop-in latency (tools/latency_pair.py) and batch-64 step (tools/b64_probe.py)
# per library variant, REPS rounds alternating; the parity subset first on
# the first non-base variant.  usage: VARIANTS="base v1" tools/gpu_latency_ab.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
VS=${VARIANTS:-base}
for v in $VS; do
  [ $v = base ] && continue
  PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
    --timeout 120 --timeout-method thread -k "lines or lsd or frame or latency or single" > gpurun_out/lat_ab_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/lat_ab_tests.log)"; [ $rc -ne 0 ] && exit $rc
  break
done
for rep in $(seq 1 ${REPS:-2}); do for v in $VS; do
  if [ $v = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  a=$(timeout -k 10 120 python -u tools/latency_pair.py 2>/dev/null | tail -1); rc=$?; [ $rc -ne 0 ] && { echo "$v latency rc=$rc"; exit $rc; }
  b=$(timeout -k 10 120 python -u tools/b64_probe.py 64 60 2>/dev/null | tail -1); rc=$?; [ $rc -ne 0 ] && { echo "$v b64 rc=$rc"; exit $rc; }
  echo "$v | $a | $b"
done; done
exit 0
