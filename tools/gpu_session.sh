#!/bin/bash
# One gpurun session: GPU tests, bench, rocprof kernel-trace stats, PMC passes.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
# Knobs: SKIP_TESTS, SKIP_BENCH, SKIP_PROF, SKIP_PMC, PYTEST_ARGS, BENCH_ARGS, PROF_ARGS.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
fatal() { case $1 in 0) ;; 124|134|137|139) echo "FATAL exit $1 in $2 — stopping"; exit $1;; *) [ "${3:-}" = hard ] && { echo "exit $1 in $2 — stopping"; exit $1; };; esac; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "== tests"
  timeout -k 10 ${TEST_T:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=8 ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -15; fatal $rc tests
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  echo "== bench"
  timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; fatal $rc bench hard
fi
PARGS=${PROF_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp
if [ "${SKIP_PROF:-0}" != 1 ]; then
  echo "== rocprof stats"
  # the bench command itself (default arguments unless STATS_ARGS is set)
  timeout -k 10 ${PROF_T:-400} rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py ${STATS_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; tail -3 $OUT/prof.log; fatal $rc rocprof hard
  python3 $R/tools/timed_stats.py $OUT/prof/run_kernel_trace.csv $OUT/kernel_stats_timed.csv
  # the bench line of the profiled run: its roofline.avg_launch_ms times the
  # same launches as kernel_stats_timed.csv (profiles/r05/prof_reps/README.md)
  grep -h '^{"metric"' $OUT/prof.log > $OUT/bench_under_rocprof.json || true
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  # calibrated HBM traffic of the roofline kernels (separate FETCH_SIZE / WRITE_SIZE passes)
  echo "== pmc traffic"
  cd $R && B=${PMC_B:-3072} bash tools/gpu_traffic.sh > $OUT/pmc.log 2>&1
  rc=$?; tail -4 $OUT/pmc.log; fatal $rc pmc hard
fi
exit 0
