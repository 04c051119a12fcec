#!/bin/bash
# r06: region2rect grid (blocks, frames, octaves) -- octave 0 of every frame
# first (in-tree) -- vs (blocks, octaves, frames) (variants/rectold)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "line or lsd or frame" > gpurun_out/r06_rectlpt_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_rectlpt_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_rectlpt_tests.log | head -20; exit $rc; }
for rep in 1 2 3; do
  for v in rectold -; do
    if [ $v = - ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-side > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    echo "[$v] $(python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline']
print(round(d['value']), round(d['ms_per_step'],2), 'frac', round(r['frac'],3), 'lines_only', d['part_fps']['lines_only'], 'grow', d['stage_ms']['lines.region_grow'], 'mism', d['oracle_check']['mismatches'])")"
  done
done
