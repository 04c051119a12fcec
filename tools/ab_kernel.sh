#!/bin/bash
# A/B of library variants on one kernel: tools/ab_kernel.sh "main v1 v2" KERNEL_SUBSTR [micro args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in $1; do
  if [ "$v" = main ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  PLVI_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ab_$v -o run --output-format csv -- python3 $R/tools/orb_micro.py ${@:3} > $OUT/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/ab_$v.log; exit 1; }
  f=$(find $OUT/ab_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep "$2" "$f" | awk -F'",' '{print $2}' | cut -d, -f1-6)"
done
