#!/bin/bash
# r06 final: tools/gpu_session.sh (GPU tests, bench, rocprofv3 stats, PMC), then the BASELINE C4 line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_session.sh || exit $?
cd $R && timeout -k 10 400 python bench.py --c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_c4.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print('c4', round(d['value']), d['ms_per_step'])"
