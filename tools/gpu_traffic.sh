#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) over tools/pmc_frame.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/traffic; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 $R/tools/pmc_frame.py ${B:-3072} 2 > $OUT/$C.log 2>&1 || { echo "pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
cd $R && python3 tools/pmc_traffic.py $OUT gpurun_out/traffic_out ${B:-3072} $((1<<30)) > gpurun_out/traffic.json && cat gpurun_out/traffic.json
find $OUT -name "*.csv" -size +20M -delete
