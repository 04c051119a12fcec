"""Diagnostic: per-launch durations of selected kernels inside bench.py's timed window
(spin_kernel markers) of a rocprofv3 kernel trace, and how much of the window each kernel
class keeps busy.  usage: python tools/kernel_spans.py run_kernel_trace.csv [label]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
timed = rows[marks[0] + 1:marks[1]]
t0 = int(timed[0]["Start_Timestamp"])
span = (max(int(r["End_Timestamp"]) for r in timed) - t0) / 1e6


def dur(pat):
    return [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 2) for r in timed
            if re.search(pat, r["Kernel_Name"])]


def busy(pat):
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in timed if re.search(pat, r["Kernel_Name"]))
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            tot, cs, ce = tot + ce - cs, s, e
    return (tot + (ce - cs if cs is not None else 0)) / 1e6


label = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"{label} timed window {span:.1f} ms")
for pat in ["orb_describe", "lsd_grow", "lsd_rect", "orb_cell_nms", "orb_blur_fast"]:
    print(f"  {pat:16s} per launch {dur(pat)}")
for pat in ["lsd_grow", "orb_", "lbd_", "lsd_rect|line_assemble"]:
    b = busy(pat)
    print(f"  busy {pat:22s} {b:8.1f} ms ({100 * b / span:4.1f} %)")
