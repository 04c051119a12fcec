#!/bin/bash
# Region-growing iteration: line parity tests (main library), then per library
# variant (VARIANTS="base main": variants/NAME or lib/) cycle stats at B=3072
# and a short bench (isolated stage times).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --maxfail=3 \
    -k "${PYTEST_K:-lines or frame or lsd}" > $OUT/it_tests.log 2>&1
  rc=$?; tail -4 $OUT/it_tests.log; [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; }
fi
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then export PLVI_LIB=""; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  echo "== $v"
  if [ "${SKIP_STATS:-0}" != 1 ]; then
    timeout -k 10 200 python tools/grow_stats.py ${STATS_B:-3072} > $OUT/it_gs_$v.txt 2>&1 || { tail -5 $OUT/it_gs_$v.txt; exit 1; }
    grep -E "octave|cycles/|per round|wave time|prefetch" $OUT/it_gs_$v.txt
  fi
  timeout -k 10 300 python bench.py --steps 10 --no-extra --no-side --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/it_bench_$v.json 2> $OUT/it_bench_$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $OUT/it_bench_$v.err; exit $rc; }
  python -c "
import json; d=json.load(open('$OUT/it_bench_$v.json')); s=d['stage_ms']
print('$v FPS', round(d['value']), 'grow', s['lines.region_grow'], 'prep', s['lines.lsd_prep'], 'lbd', s['lines.lbd'], 'orb_blur', s['orb.level'], 'check', d.get('oracle_check',{}).get('mismatches'), d.get('failed'))"
done
