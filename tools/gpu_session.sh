#!/bin/bash
# One gpurun session: GPU tests, bench, rocprof kernel-trace stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL exit $1 in $2 — stopping"; exit $1;; esac; }

echo "== tests"
timeout -k 10 ${TEST_T:-900} python -m pytest tests -m gpu -q --maxfail=8 ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
rc=$?; tail -30 $OUT/gpu_tests.log; fatal $rc tests
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
echo "== bench"
timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; fatal $rc bench
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
echo "== rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_T:-400} rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; tail -3 $OUT/prof.log; fatal $rc rocprof
find $OUT/prof -name "*stats*" | head
exit 0
