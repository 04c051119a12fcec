#!/bin/bash
# Address-translation counters of the region-growing kernel at B = 3072: the
# TCP UTCL1 translation hit / miss counters available on this box (names from
# rocprofv3 --list-avail), one pass, for the in-tree library and LIBS variants.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
C=""
for n in TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum; do
  grep -qE "Counter_Name[[:space:]]*:[[:space:]]*$n\$" $OUT/avail.txt && C="$C $n"
done
echo "counters: $C"
[ -z "$C" ] && exit 0
for v in main ${LIBS:-}; do
  if [ $v = main ]; then L=""; else L=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  PMC_SETS="$C" PMC_CMD="tools/lines_micro.py 3072 2" KSHOW=lsd_grow LIBV=$L bash $R/tools/gpu_pmc_k.sh > /dev/null || exit 1
  echo "== $v"; grep -A4 "lsd_grow" $OUT/pmc_k_table.txt | head -6
done
