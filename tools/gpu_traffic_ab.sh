#!/bin/bash
# ORB tests, then traffic + isolated ORB kernel times for the main library and variants (VARIANTS="a32 ...")
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x -k "${PYTEST_K:-orb and not stereo}" > gpurun_out/t.log 2>&1
rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
for v in main ${VARIANTS:-}; do
  if [ $v = main ]; then export PLVI_LIB=; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"
  bash tools/gpu_traffic.sh > gpurun_out/traffic_$v.log 2>&1 || { echo traffic failed; tail -5 gpurun_out/traffic_$v.log; exit 1; }
  cp gpurun_out/traffic.json gpurun_out/traffic_$v.json
  python3 -c "
import json
for e in json.load(open('gpurun_out/traffic_$v.json')):
    print(e['kernel'], 'fetch %.3e write %.3e total %.3e' % (e['fetch_bytes'], e['write_bytes'], e['bytes_per_launch']))"
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ok_$v -o run --output-format csv -- python3 $R/tools/orb_micro.py 3072 3 > $R/gpurun_out/ok_$v.log 2>&1) || { echo prof failed; exit 1; }
  python3 tools/ktimes.py $(find gpurun_out/ok_$v -name "*kernel_stats.csv" | head -1) | head -4
  find gpurun_out/ok_$v -name "*kernel_trace.csv" -delete
done
