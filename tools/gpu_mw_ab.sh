#!/bin/bash
# A/B of region-growing variants (tools/build_variant.sh): mw_probe at B=1,64
# and the batch-64 step, per variant (default = the in-tree library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in default ${VARIANTS:-}; do
  if [ $v = default ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v" >> $OUT/mw_ab.log
  PLVI_LIB=$L timeout -k 10 150 python tools/mw_probe.py 1,64 2>&1 | grep "mw=256" | cut -c1-400 >> $OUT/mw_ab.log || exit $?
  PLVI_LIB=$L timeout -k 10 120 python tools/b64_probe.py 64 20 2>&1 | grep FPS >> $OUT/mw_ab.log || exit $?
  PLVI_LIB=$L timeout -k 10 120 python tools/latency_probe.py 2>&1 | grep median >> $OUT/mw_ab.log || exit $?
done
