#!/bin/bash
# PMC table of the line extractor run alone (tools/lines_micro.py), one pass per counter set
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
S2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_LDS_IDX_ACTIVE"
PMC_SETS="${PMC_SETS:-$S1;$S2}" PMC_CMD="tools/lines_micro.py ${B:-3072} 2" KSHOW=${KSHOW:-lsd_prep} bash $R/tools/gpu_pmc_k.sh && cp $R/gpurun_out/pmc_k_table.txt $R/gpurun_out/pmc_lines_table.txt
