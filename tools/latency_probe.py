"""Single-frame latency (host image in, host tables out) of plvi_lines_extract
and plvi_orb_extract, median of 30, and the lines-only batch-16 stage time."""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

imgs = [synth.frame(s) for s in range(10)]
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480)
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480)
for im in imgs[:3]:
    lx(im)
    orb(im)
tl, to = [], []
for k in range(30):
    im = imgs[k % 10]
    t = time.perf_counter()
    lx(im)
    tl.append(time.perf_counter() - t)
    t = time.perf_counter()
    orb(im)
    to.append(time.perf_counter() - t)
print(f"lines median {np.median(tl) * 1e3:.2f} ms  orb median {np.median(to) * 1e3:.2f} ms")
