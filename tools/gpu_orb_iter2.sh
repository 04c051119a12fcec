#!/bin/bash
# ORB iteration: ORB GPU tests, then isolated kernel times + one SQ PMC pass (tools/gpu_orb_prof.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x -k "${PYTEST_K:-orb and not stereo}" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
PMC_SETS="${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR}" bash tools/gpu_orb_prof.sh > $OUT/op.log 2>&1
rc=$?; python3 tools/ktimes.py $OUT/orbk/run_kernel_stats.csv; grep -A12 "^${KSHOW:-orb_blur_fast}" $OUT/pmc_k_table.txt; exit $rc
