"""Print average per-kernel durations (ms) of the plvi kernels in a rocprofv3 kernel_stats.csv."""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
    if "plvi" in n:
        print(f"{n:44s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e6:9.3f} ms")
