#!/bin/bash
# r04 measurement session: default bench line, rocprofv3 kernel trace of the
# same command (timed-window stats + step timeline), calibrated HBM traffic
# passes, orb_describe PMC (alone / in the schedule).  Each GPU step has its
# own time limit; the first failure ends the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > $OUT/bench_r04.json 2> $OUT/bench_r04.err || { echo "bench failed"; tail -20 $OUT/bench_r04.err; exit 1; }
  cut -c1-400 $OUT/bench_r04.json
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline ${PROF_ARGS:---steps 6 --warmup 2 --no-extra --no-side} > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
  cd $R
  T=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
  python3 tools/timed_stats.py $T $OUT/kernel_stats_timed.csv && head -25 $OUT/kernel_stats_timed.csv | cut -c1-150
  python3 tools/step_timeline.py $T > $OUT/step_timeline.txt; cat $OUT/step_timeline.txt
  S=$(find $OUT/prof -name "run_kernel_stats.csv" | head -1); cp $S $OUT/kernel_stats.csv
  find $OUT/prof -name "*.csv" -size +20M -delete
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  B=${PMC_B:-3072} bash tools/gpu_traffic.sh > $OUT/traffic.log 2>&1 || { echo "traffic failed"; tail -8 $OUT/traffic.log; exit 1; }
  tail -40 $OUT/traffic.log | grep -E "kernel|bytes_per_launch"
fi
if [ "${SKIP_DESC:-0}" != 1 ]; then
  bash tools/gpu_pmc_describe.sh > $OUT/pmc_desc.log 2>&1 || { echo "describe pmc failed"; tail -8 $OUT/pmc_desc.log; exit 1; }
  cat $OUT/pmc_desc.log | head -60
fi
