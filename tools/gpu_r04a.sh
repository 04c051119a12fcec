#!/bin/bash
# r04 first session: grow PMC tables, mw memory-model A/B, default bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
bash tools/gpu_pmc_grow.sh > $OUT/pmc_grow.log 2>&1 || { echo "pmc grow failed"; tail -20 $OUT/pmc_grow.log; exit 1; }
echo "pmc grow ok"
VARIANTS="mwrelaxed" bash tools/gpu_mw_ab.sh || { echo "mw ab failed"; cat $OUT/mw_ab.log; exit 1; }
cat $OUT/mw_ab.log | cut -c1-300
timeout -k 10 400 python bench.py > $OUT/bench_r04a.json 2> $OUT/bench_r04a.err || { echo bench failed; tail -20 $OUT/bench_r04a.err; exit 1; }
cut -c1-600 $OUT/bench_r04a.json
