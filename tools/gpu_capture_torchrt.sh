#!/bin/bash
# The capture diagnostics on PyTorch's bundled HIP runtime (torch/lib, the one
# a process that imports torch first maps) instead of /opt/rocm's; the frame
# capture runs last.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TL=$(python -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
for v in 0 1 2 3 4 5 6; do
  LD_LIBRARY_PATH=$TL timeout -k 10 60 $R/tools/_build/capture_probe $v >> $OUT/capture_probe_torchrt.log 2>&1
  rc=$?; echo "variant $v rc=$rc" >> $OUT/capture_probe_torchrt.log
  case $rc in 0|1) ;; *) echo "probe variant $v exit $rc: stopping"; exit $rc;; esac
done
LD_LIBRARY_PATH=$TL timeout -k 10 120 $R/tools/_build/capture_frame 16 1 0 > $OUT/capture_frame_torchrt.log 2>&1
rc=$?; echo "capture_frame rc=$rc" >> $OUT/capture_frame_torchrt.log
exit $rc
