#!/bin/bash
# Variant check: parity tests (-k PYTEST_K) and calibrated PMC traffic with
# variants/$V, then a bench sweep of main vs the variant.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=$R/pl-vi-orbslam3_amd/variants/$V/libplvi_frontend.so
PLVI_LIB=$L timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --maxfail=3 -k "${PYTEST_K:-orb or frame}" > gpurun_out/vc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/vc_tests.log; [ $rc -ne 0 ] && exit $rc
PLVI_LIB=$L B=3072 bash tools/gpu_traffic.sh > gpurun_out/vc_pmc.log 2>&1 || { tail -5 gpurun_out/vc_pmc.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/traffic.json'))
for e in d: print('$V', e['kernel'], round(e['fetch_bytes']/1e9,3), round(e['write_bytes']/1e9,3), round(e['bytes_per_launch']/1e9,3))"
SWEEP="X=1
PLVI_LIB=$L" bash tools/gpu_sched_sweep.sh
