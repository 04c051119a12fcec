"""Per-kernel table of PMC counters from tools/pmc_session.sh output (diagnostic).
usage: python tools/pmc_table.py gpurun_out/pmc_orb"""
import csv
import pathlib
import re
import sys
from collections import defaultdict

d = pathlib.Path(sys.argv[1])
agg = defaultdict(lambda: defaultdict(float))
ndisp = defaultdict(set)
for f in sorted(d.glob("p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("plvi::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ndisp[(k, f.parent.name)].add(r["Dispatch_Id"])
cols = sorted({c for v in agg.values() for c in v})
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    print(k)
    for c in cols:
        if c in v:
            print(f"   {c:24s} {v[c]:16.0f}")
    if v.get("SQ_WAVES"):
        w = v["SQ_WAVES"]
        print(f"   per wave: cycles(x4) {4*v.get('SQ_WAVE_CYCLES',0)/w:9.0f}  valu {v.get('SQ_INSTS_VALU',0)/w:7.0f}  "
              f"lds {v.get('SQ_INSTS_LDS',0)/w:6.0f}  wait_any {4*v.get('SQ_WAIT_ANY',0)/w:8.0f}  "
              f"wait_inst {4*v.get('SQ_WAIT_INST_ANY',0)/w:8.0f}  active {4*v.get('SQ_ACTIVE_INST_ANY',0)/w:8.0f}")
