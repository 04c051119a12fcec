"""Diagnostic: kernel timeline of one timed step (bench.py spin_kernel markers).
usage: python tools/step_timeline.py run_kernel_trace.csv [step]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
timed = rows[marks[0] + 1:marks[1]]
# one slot's period: from one of its lsd_half launches to its next (the
# other slot's launches fall in between with two batches in flight)
halves = [i for i, r in enumerate(timed) if "lsd_half_kernel" in r["Kernel_Name"]]
q0 = timed[halves[0]]["Queue_Id"]
starts = [i for i in halves if timed[i]["Queue_Id"] == q0]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
i0, i1 = starts[k], starts[k + 1] if k + 1 < len(starts) else len(timed)
t0 = int(timed[i0]["Start_Timestamp"])
for r in timed[i0:i1]:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("plvi::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{name[:34]:34s} q{r['Queue_Id']:>3s} {s:8.2f} {e:8.2f} {e - s:7.2f}")
