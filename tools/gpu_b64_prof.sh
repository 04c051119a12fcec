#!/bin/bash
# batch-64 step timeline: rocprofv3 kernel trace of tools/b64_probe.py
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 120 python $R/tools/b64_probe.py ${B:-64} 10 > $OUT/b64_plain.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/b64prof -o run --output-format csv -- python3 $R/tools/b64_probe.py ${B:-64} 10 > $OUT/b64_prof.log 2>&1 || exit $?
python3 $R/tools/step_timeline.py $OUT/b64prof/run_kernel_trace.csv > $OUT/b64_timeline.txt
