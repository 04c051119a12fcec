"""Per-queue busy time and per-kernel mean durations in bench.py's timed window
(between the spin_kernel markers) of a rocprofv3 kernel trace.
usage: python tools/queue_busy.py run_kernel_trace.csv"""
import csv, re, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
timed = rows[marks[0] + 1:marks[1]]
t0 = int(timed[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in timed)
q = collections.defaultdict(list)
for r in timed:
    q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("plvi::", "")))
W = (t1 - t0) / 1e6
print(f"window {W:.1f} ms")
for k, v in sorted(q.items()):
    busy = sum(e - s for s, e, _ in v) / 1e6
    names = collections.Counter(n.split("<")[0] for _, _, n in v)
    print(f"q{k:>3s} busy {busy:7.1f} ms ({100*busy/W:5.1f} %) launches {len(v):4d} {dict(names)}")
print()
for k, v in sorted(q.items()):
    d = collections.defaultdict(list)
    for s_, e_, n in v: d[n.split("<")[0]].append((e_ - s_) / 1e6)
    print(f"q{k}: " + ", ".join(f"{n.replace('orb_','').replace('_kernel','')} {sum(x)/len(x):.1f}" for n, x in d.items()))
