"""Diagnostic: cycle accounting of the LSD region-growing kernel on one batch."""
import sys, pathlib, numpy as np
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi
from plvi import synth
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
frames = synth.batch(B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
buf = plvi.DeviceBuffer(frames.nbytes); buf.upload(frames)
st = plvi.DeviceBuffer(B * 2 * 16 * 8)
lib = plvi.load()
lx.extract_batch(buf.ptr, B, 640 * 480, 640); lib.plvi_device_synchronize()
lib.plvi_lines_debug_stats(lx._h, __import__("ctypes").c_void_p(st.ptr))
lx.extract_batch(buf.ptr, B, 640 * 480, 640); lib.plvi_device_synchronize()
s = st.download(np.zeros((B, 2, 16), np.uint64)).astype(np.float64)
names = ["total", "block_setup", "rounds", "rect", "seeds", "blocks", "rounds_n", "rect_pts", "commits", "ph_decide", "ph_angles", "ph_verify", "ph_commit"]
for o in range(2):
    print(f"octave {o}:")
    for i, n in enumerate(names):
        print(f"  {n:10s} mean {s[:, o, i].mean():14.0f}  max {s[:, o, i].max():14.0f}")
    t = s[:, o]
    print("  setup cycles/block %.0f  round cycles/round %.0f  rounds/block %.2f  commits/round %.2f  rect cycles/pt %.0f  total cycles/commit %.0f" % (
        (t[:, 1] / t[:, 5]).mean(), (t[:, 2] / t[:, 6]).mean(), (t[:, 6] / t[:, 5]).mean(), (t[:, 8] / t[:, 6]).mean(),
        (t[:, 3] / np.maximum(t[:, 7], 1)).mean(), (t[:, 0] / np.maximum(t[:, 8], 1)).mean()))
    print("  per round: decide %.0f  angles %.0f  verify %.0f  commit %.0f" % tuple((t[:, 9 + k] / t[:, 6]).mean() for k in range(4)))
