#!/bin/bash
# rocprofv3 kernel-trace passes of the default bench command, REPS times: the
# timed-window stats of each (tools/timed_stats.py) plus the per-launch
# durations of the roofline kernels; the large traces are deleted.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 ${REPS:-2}); do
  rm -rf $OUT/profrep
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/profrep -o run --output-format csv -- python3 $R/bench.py > $OUT/profrep_$i.log 2>&1 || { echo "rep $i failed"; tail -3 $OUT/profrep_$i.log; exit 1; }
  python3 $R/tools/timed_stats.py $OUT/profrep/run_kernel_trace.csv $OUT/kst_rep$i.csv > /dev/null
  cp $OUT/profrep/run_kernel_stats.csv $OUT/ks_rep$i.csv
  python3 - $OUT/profrep/run_kernel_trace.csv $OUT/launches_rep$i.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
m = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
with open(sys.argv[2], "w") as f:
    for k in ("orb_blur_fast_kernel", "orb_pyramid_kernel", "lsd_grow_kernel"):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[m[0] + 1:m[1]] if k in r["Kernel_Name"]]
        f.write(f"{k}: mean {sum(d) / len(d):.2f} ms over {len(d)}: " + " ".join(f"{x:.1f}" for x in d) + "\n")
PY
  python3 -c "import json;d=json.load(open('$OUT/profrep_$i.log'.replace('.log','.log'))) " 2>/dev/null
  grep -h '"value"' $OUT/profrep_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('rep', $i, 'bench value', round(d['value']), 'roofline avg_launch_ms', round(d['roofline']['avg_launch_ms'],2))" || true
  cat $OUT/launches_rep$i.txt
  rm -rf $OUT/profrep
done
