#!/bin/bash
# A/B of ORB variants (tools/build_variant.sh): per-stage times at B=3072
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in default ${VARIANTS:-}; do
  if [ $v = default ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v" >> $OUT/orb_ab.log
  PLVI_LIB=$L timeout -k 10 120 python tools/orb_stages.py ${B:-3072} 5 2>&1 | grep FPS >> $OUT/orb_ab.log || exit $?
done
