#!/bin/bash
# One PMC pass per counter set over tools/orb_micro.py; per-kernel table (tools/pmc_table.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_k
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL}"
for C in "${SETS[@]}"; do
  i=$((i+1))
  PLVI_LIB=${LIBV:-} timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 $R/${PMC_CMD:-tools/orb_micro.py 3072 2} > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_table.py $OUT > $R/gpurun_out/pmc_k_table.txt; grep -A16 "${KSHOW:-orb_pyramid}" $R/gpurun_out/pmc_k_table.txt || true; rm -rf $OUT
