#!/bin/bash
# batch-64 step with and without 3072-frame handles present, queue settings,
# and the kernel trace's hardware-queue ids of the --big case
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
{
timeout -k 10 100 python tools/b64_probe.py 64 20 || exit $?
timeout -k 10 100 python tools/b64_probe.py 64 20 --big || exit $?
PLVI_ORB_PRIO=0 timeout -k 10 100 python tools/b64_probe.py 64 20 --big || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 100 python tools/b64_probe.py 64 20 --big || exit $?
} 2>&1 | grep -v amdgpu.ids > $OUT/b64q.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/b64bigprof -o run --output-format csv -- python3 $R/tools/b64_probe.py 64 10 --big > $OUT/b64big_prof.log 2>&1 || exit $?
python3 $R/tools/step_timeline.py $OUT/b64bigprof/run_kernel_trace.csv > $OUT/b64big_timeline.txt
