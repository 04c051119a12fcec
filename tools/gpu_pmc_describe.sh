#!/bin/bash
# orb_describe_kernel PMC alone (tools/orb_micro.py) and
# inside the frame schedule (tools/pmc_frame.py), one rocprofv3 run per pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_desc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/counters.txt 2>&1 || true
pick() { grep -oE "\b$1\b" $OUT/counters.txt | head -1; }
TA=$(pick "TA_BUSY_avr|TA_TA_BUSY_sum|TA_BUSY_sum"); TD=$(pick "TD_BUSY_avr|TD_TD_BUSY_sum|TD_BUSY_sum")
LV=$(pick "SQ_LEVEL_WAVES"); echo "TA=$TA TD=$TD LV=$LV"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
S2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU $LV TCC_HIT_sum TCC_MISS_sum $TA $TD"
for cfg in "iso:tools/orb_micro.py 3072 2" "sched:tools/pmc_frame.py 3072 2"; do
  name=${cfg%%:*}; cmd=${cfg#*:}
  PMC_SETS="$S1;$S2" PMC_CMD="$cmd" KSHOW=orb_describe bash $R/tools/gpu_pmc_k.sh > /dev/null || { echo "pmc $name failed"; exit 1; }
  cp $R/gpurun_out/pmc_k_table.txt $OUT/pmc_describe_$name.txt
  echo "== $name"; grep -A24 "orb_describe" $OUT/pmc_describe_$name.txt | head -26
done
