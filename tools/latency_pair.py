"""Drop-in single-frame latency as bench.py measures it (ORB || lines on two
host threads, host image in, host tables out), median over 24 frames, in a
fresh process that holds only these two extractors, as a SLAM process does
(bench.py runs it as a child: its own process holds ~20 more handles whose
streams share the runtime's hardware queues).  --json: one JSON line."""
import json
import pathlib
import sys
import threading
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

imgs = [synth.frame(s) for s in range(24)]
sl = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480)
so = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480)
lat, lo_, ll_ = [], [], []
for rep in range(len(imgs) + 6):
    img = imgs[rep % len(imgs)]
    res = {}

    def ro():
        t = time.perf_counter()
        so(img)
        res["orb"] = time.perf_counter() - t

    def rl():
        t = time.perf_counter()
        sl(img)
        res["lines"] = time.perf_counter() - t
    t0 = time.perf_counter()
    th = [threading.Thread(target=ro), threading.Thread(target=rl)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if rep >= 6:
        lat.append(time.perf_counter() - t0)
        lo_.append(res["orb"])
        ll_.append(res["lines"])
if "--json" in sys.argv:
    print(json.dumps({"median_ms": float(np.median(lat)) * 1e3, "p90_ms": float(np.percentile(lat, 90)) * 1e3,
                      "orb_median_ms": float(np.median(lo_)) * 1e3, "lines_median_ms": float(np.median(ll_)) * 1e3,
                      "frames": len(lat)}), flush=True)
    sys.exit(0)
print(f"pair median {np.median(lat) * 1e3:.2f} ms p90 {np.percentile(lat, 90) * 1e3:.2f} | "
      f"orb {np.median(lo_) * 1e3:.2f} lines {np.median(ll_) * 1e3:.2f}", flush=True)
