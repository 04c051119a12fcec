"""Diagnostic: per-step kernel timeline from a rocprofv3 kernel trace CSV.
usage: python tools/timeline.py run_kernel_trace.csv [step_index]
Steps are delimited by the ORB pyramid launches (one per step)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
rows = [r for r in rows if "plvi::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "orb_pyramid_kernel" in r["Kernel_Name"]]
i0 = starts[k]
i1 = starts[k + 1] if k + 1 < len(starts) and k != -1 else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("plvi::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{name:34s} q{r['Queue_Id']:>3s} {s:8.2f} {e:8.2f} {e - s:7.2f}")
