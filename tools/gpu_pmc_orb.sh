#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pmc_orb/stats -o run --output-format csv -- python3 $R/tools/orb_micro.py 3072 5 > $OUT/pmc_orb_stats.log 2>&1 || exit $?
f=$(find $OUT/pmc_orb/stats -name "*kernel_stats.csv" | head -1); cut -c1-160 "$f" | head -12
i=0
for C in "${PMC_SETS[@]:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_orb/p$i -o run --output-format csv -- python3 $R/tools/orb_micro.py 3072 2 > $OUT/pmc_orb_p$i.log 2>&1 || exit $?
done
python3 $R/tools/pmc_table.py $OUT/pmc_orb 2>/dev/null | head -40 || true
