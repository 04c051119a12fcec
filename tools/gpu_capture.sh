#!/bin/bash
# graph-capture diagnostics (built by tools/build_capture.sh); the frame
# capture runs last: a crash there ends the call
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for v in 0 1 2 3 4 5 6; do
  timeout -k 10 60 $R/tools/_build/capture_probe $v >> $OUT/capture_probe.log 2>&1
  rc=$?; echo "variant $v rc=$rc" >> $OUT/capture_probe.log
  case $rc in 0|1) ;; *) echo "probe variant $v exit $rc: stopping"; exit $rc;; esac
done
timeout -k 10 120 $R/tools/_build/capture_frame ${CAP_N:-16} 1 ${CAP_MODE:-0} > $OUT/capture_frame.log 2>&1
rc=$?; echo "capture_frame rc=$rc" >> $OUT/capture_frame.log; cat $OUT/capture_frame.log
exit $rc
