#!/bin/bash
# r06: octree phase-2 rank sort -- ORB / frame / stereo parity, then the bench
# (stage_ms: orb.octree alone; the step)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or scale or stereo or c4" > gpurun_out/r06_oct_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_oct_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/oct_bench.json 2> gpurun_out/oct_bench.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/oct_bench.err; exit $rc; }
python3 -c "
import json;d=json.load(open('gpurun_out/oct_bench.json'))
print(round(d['value']), round(d['ms_per_step'],2), d['stage_ms'], d['part_fps'], 'b64', round(d['batch64']['value']), 'lat', round(d['single_frame_latency']['drop_in_process']['median_ms'],2), d['oracle_check'])"
