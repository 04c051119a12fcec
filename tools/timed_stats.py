"""Per-kernel statistics of bench.py's timed region from a rocprofv3 kernel trace.

bench.py launches a `spin_kernel` (torch.cuda._sleep) right before and right
after its timed region; the kernels that start between the two markers are
exactly the timed steps' launches, i.e. the launch set the bench's own HIP
events average for `roofline.avg_launch_ms`.  Writes a kernel-stats CSV
(rocprofv3 column names) for that window.

usage: python tools/timed_stats.py run_kernel_trace.csv out.csv
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("timed_stats: no spin_kernel markers in the trace")
    a, b = marks[0], marks[1]
    t_lo, t_hi = int(rows[a]["End_Timestamp"]), int(rows[b]["Start_Timestamp"])
    agg = defaultdict(list)
    for r in rows[a + 1:b]:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        agg[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values())
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
    print(f"timed window {(t_hi - t_lo) / 1e6:.2f} ms, {b - a - 1} launches")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"  {n[:48]:48s} {len(v):5d} x {sum(v) / len(v) / 1e6:8.3f} ms")


if __name__ == "__main__":
    main()
