#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) over tools/pmc_frame.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/traffic; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 $R/tools/pmc_frame.py ${B:-3072} 2 > $OUT/$C.log 2>&1 || { echo "pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
# instruction counts (4 SQ counters: one pass)
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $OUT/pmc_VALU -o run --output-format csv -- python3 $R/tools/pmc_frame.py ${B:-3072} 2 > $OUT/VALU.log 2>&1 || { echo "pass VALU failed"; tail -5 $OUT/VALU.log; exit 1; }
cd $R && python3 tools/pmc_traffic.py $OUT gpurun_out/traffic_out ${B:-3072} $((1<<30)) > gpurun_out/traffic.json && cat gpurun_out/traffic.json
find $OUT -name "*.csv" -size +20M -delete
