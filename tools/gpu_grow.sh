#!/bin/bash
# region-growing iteration: grow-window tests, a window sweep at B (SWEEP), optional bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -x -k "${PYTEST_K:-grow_window or lines_golden or lines_batch}" > $OUT/grow_tests.log 2>&1
rc=$?; tail -3 $OUT/grow_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/grow_sweep.py "${SWEEP:-6144:2,6144:64,6144:32,6144:128,12288:64:2}" "${SWEEP_B:-3072}" > $OUT/grow_sweep.txt 2>&1
rc=$?; cat $OUT/grow_sweep.txt; [ $rc -ne 0 ] && exit $rc
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --no-side > $OUT/bench_g.json 2> $OUT/bench_g.err
  rc=$?; cut -c1-300 $OUT/bench_g.json; python -c "import json;d=json.load(open('$OUT/bench_g.json'));print(d['stage_ms'],d['part_fps'],d['oracle_check'])"; exit $rc
fi
