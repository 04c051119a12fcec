#!/bin/bash
# round-2 session A: GPU tests, default bench, C4 bench (world 1, gather path exercised)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=12 > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -20
case $rc in 0|1) ;; *) echo "tests rc=$rc, stopping"; exit $rc;; esac
echo "== bench"
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err
case $rc in 0|1) ;; *) echo "bench rc=$rc, stopping"; exit $rc;; esac
echo "== bench c4"
timeout -k 10 400 python bench.py --c4 --gather --steps 10 --no-cpu-baseline --no-side --no-extra > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?; cat $OUT/bench_c4.json; tail -5 $OUT/bench_c4.err
exit $rc
