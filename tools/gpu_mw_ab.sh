#!/bin/bash
# multi-wave growth A/B: parity subset per variant, then tools/mw_probe.py per variant.
# usage: VARIANTS="base pf warm" tools/gpu_mw_ab.sh   (base = the in-tree library)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
      -k "${PYTEST_K:-lines or lsd or grow or frame}" > $OUT/mw_ab_tests_$v.log 2>&1
    rc=$?; echo "$v tests: $(tail -1 $OUT/mw_ab_tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
  fi
  timeout -k 10 240 python -u tools/mw_probe.py ${MWB:-1,64} > $OUT/mw_ab_$v.txt 2>&1
  rc=$?; echo "== $v"; grep -v amdgpu.ids $OUT/mw_ab_$v.txt | cut -c1-330; [ $rc -ne 0 ] && exit $rc
done
exit 0
