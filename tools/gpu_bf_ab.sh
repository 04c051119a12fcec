set -u
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --maxfail=3 -k "orb or frame" > gpurun_out/bf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bf_tests.log; [ $rc -ne 0 ] && exit $rc
SWEEP="PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/bf0/libplvi_frontend.so
X=1
PLVI_GROW_AFTER_BLUR=0" bash tools/gpu_sched_sweep.sh
