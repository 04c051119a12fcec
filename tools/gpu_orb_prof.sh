#!/bin/bash
# ORB extractor alone: kernel trace stats + PMC passes (tools/gpu_pmc_k.sh) on tools/orb_micro.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rm -rf $OUT/orbk
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/orbk -o run --output-format csv -- python3 $R/tools/orb_micro.py 3072 3 > $OUT/orbk.log 2>&1 || { tail -5 $OUT/orbk.log; exit 1; }
f=$(find $OUT/orbk -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | sed 's/(.*)"/"/' | head -14
rm -f $(find $OUT/orbk -name "*kernel_trace.csv")
cd $R && PMC_SETS="${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;FETCH_SIZE;WRITE_SIZE}" PMC_CMD="tools/orb_micro.py 3072 2" KSHOW=${KSHOW:-orb_blur_fast} bash tools/gpu_pmc_k.sh
