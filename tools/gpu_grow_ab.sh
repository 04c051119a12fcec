#!/bin/bash
# large-batch region growing A/B: parity subset per variant, then tools/grow_sweep.py at B (default 3072).
# usage: VARIANTS="base gpf" tools/gpu_grow_ab.sh   (base = the in-tree library)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
      -k "${PYTEST_K:-lines or lsd or grow or frame}" > $OUT/grow_ab_tests_$v.log 2>&1
    rc=$?; echo "$v tests: $(tail -1 $OUT/grow_ab_tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
  fi
  timeout -k 10 240 python -u tools/grow_sweep.py ${SWEEP:-6144} ${SWEEP_B:-3072} > $OUT/grow_ab_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -v amdgpu.ids $OUT/grow_ab_$v.txt | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
exit 0
