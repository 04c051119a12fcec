#!/bin/bash
# Run "NAME|TIMEOUT|COMMAND" steps in order, each under its own time limit,
# output to gpurun_out/NAME.log.  A test failure (exit 1) does not stop the
# sequence; a crash, abort or time limit (any other non-zero exit) does.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
worst=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 $t bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "step $name rc=$rc" | tee -a $OUT/steps.log
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -gt 1 ]; then echo "stopping after $name (exit $rc)"; exit $rc; fi
done
exit $worst
