#!/bin/bash
# PMC passes over tools/prof_stage.py (diagnostic).  STAGE=orb|lines|frame,
# PASSES="CTR CTR ...;CTR ..." (one rocprofv3 run per ';'-separated pass).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${STAGE:-orb}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
DEF="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
IFS=';' read -ra SETS <<< "${PASSES:-$DEF}"
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/prof_stage.py ${STAGE:-orb} ${B:-1024} 1 > $OUT/p$i.log 2>&1
  rc=$?; tail -1 $OUT/p$i.log; [ $rc = 0 ] || exit $rc
done
exit 0
