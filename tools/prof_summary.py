"""Summarise a gpu_session.sh run: per-kernel rocprofv3 stats + PMC bytes.

usage: python tools/prof_summary.py gpurun_out [frames_per_launch]

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.
MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced streaming read (16 B/lane); other widths are uncalibrated.  Both the
raw value and the x2-corrected fetch are printed; the JSON line (last line)
is what bench.py's `roofline.traffic` cites.
"""
import csv
import json
import pathlib
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("plvi::", "")
    return name


def pmc(path, counter):
    agg = defaultdict(list)
    f = pathlib.Path(path) / f"pmc_{counter}" / "run_counter_collection.csv"
    if not f.exists():
        return agg
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main():
    out = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    stats = {}
    for r in csv.DictReader(open(out / "prof" / "run_kernel_stats.csv")):
        stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]), float(r["Percentage"]))
    fe, wr = pmc(out, "FETCH_SIZE"), pmc(out, "WRITE_SIZE")
    print(f"{'kernel':34s} {'calls':>5s} {'avg_us':>9s} {'%':>6s} {'fetch_B/frame':>14s} {'write_B/frame':>14s}")
    res = {}
    for k, (c, avg, pct) in sorted(stats.items(), key=lambda kv: -kv[1][1] * kv[1][0]):
        f = sum(fe.get(k, [])) / max(1, len(fe.get(k, [])))
        w = sum(wr.get(k, [])) / max(1, len(wr.get(k, [])))
        print(f"{k:34s} {c:5d} {avg / 1e3:9.1f} {pct:6.2f} {f / frames:14.0f} {w / frames:14.0f}")
        res[k] = {"calls": c, "avg_ns": avg, "fetch_B_per_launch_raw": f, "write_B_per_launch": w}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
