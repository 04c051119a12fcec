#!/bin/bash
# r06: NMS survivors as candidate lists (no candidate plane / SAT / node-best
# kernels): the ORB / frame / stereo / scale parity subset, then the bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "orb or frame or scale or stereo or c4 or vocab or bow" > gpurun_out/r06_clist_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06_clist_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06_clist_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/clist_bench.json 2> gpurun_out/clist_bench.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/clist_bench.err; exit $rc; }
python3 -c "
import json;d=json.load(open('gpurun_out/clist_bench.json'))
print(round(d['value']), round(d['ms_per_step'],2), d['stage_ms'], d['part_fps'], 'b64', round(d['batch64']['value']), 'lat', round(d['single_frame_latency']['drop_in_process']['median_ms'],2), d['oracle_check'], 'bf', round(d['roofline']['avg_launch_ms'],2), round(d['roofline']['frac'],3))"
