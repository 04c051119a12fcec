#!/bin/bash
# quick loop: selected GPU tests (PYTEST_K), bench (BENCH_ARGS), optional rocprof stats (PROF=1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=5 -k "$PYTEST_K" > $OUT/gpu_tests_q.log 2>&1
  rc=$?; tail -15 $OUT/gpu_tests_q.log
  [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_q.json 2> $OUT/bench_q.err
  rc=$?; cat $OUT/bench_q.json; tail -3 $OUT/bench_q.err
  [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
fi
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_q -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-side} > $OUT/prof_q.log 2>&1
  rc=$?; tail -2 $OUT/prof_q.log
  f=$(find $OUT/prof_q -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -14 "$f" | cut -c1-200
  exit $rc
fi
