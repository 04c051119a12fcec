#!/bin/bash
# PMC tables of the two region-growing kernels (lsd_grow_kernel at B=3072,
# lsd_grow_mw_kernel at B=64 and B=1) over tools/lines_micro.py, one rocprofv3
# run per counter set, plus tools/grow_stats.py's per-block cycle split.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_grow
mkdir -p $OUT
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
S2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum"
for B in ${BS:-3072 64 1}; do
  PMC_SETS="$S1;$S2" PMC_CMD="tools/lines_micro.py $B 2" KSHOW=lsd_grow bash $R/tools/gpu_pmc_k.sh > /dev/null || exit 1
  cp $R/gpurun_out/pmc_k_table.txt $OUT/pmc_lines_B$B.txt
  echo "== B=$B"; grep -A22 "lsd_grow" $OUT/pmc_lines_B$B.txt | head -50
done
cd $R
timeout -k 10 120 python -u tools/grow_stats.py ${GS_B:-3072} > $OUT/grow_stats_B3072.txt 2>&1 || exit 1
cat $OUT/grow_stats_B3072.txt
