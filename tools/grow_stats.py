"""Diagnostic: cycle accounting of the LSD region-growing kernel on one batch
(the bench's device sequence, so B = 3072 shows the contended per-wave times).
usage: python tools/grow_stats.py [B]"""
import ctypes
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
seq = synth.device_sequence(B, 640, 480, seed=0, device="cuda:0")
torch.cuda.synchronize()
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
st = torch.zeros(B * 2 * 16, dtype=torch.int64, device="cuda:0")
lib = plvi.load()
lx.extract_batch(seq.data_ptr(), B, 640 * 480, 640)
lib.plvi_device_synchronize()
lib.plvi_lines_debug_stats(lx._h, ctypes.c_void_p(st.data_ptr()))
lx.extract_batch(seq.data_ptr(), B, 640 * 480, 640)
lib.plvi_device_synchronize()
lib.plvi_lines_debug_stats(lx._h, ctypes.c_void_p(0))
s = st.cpu().numpy().reshape(B, 2, 16).astype(np.float64)
names = ["total", "block_setup", "rounds", "rect", "seeds", "blocks", "rounds_n", "rect_pts", "commits", "ph_decide",
         "ph_angles", "ph_verify", "ph_commit", "seed_scan", "seed_start", "init"]
# 64-pixel chunks of the seed scan per octave (octave 0 = 0.8 x 640 x 480, octave 1 half of it)
dims = [(512, 384), (256, 192)]
names_chunks = [((w - 1 + 63) // 64) * (h - 1) for w, h in dims]
print(f"B = {B}")
for o in range(2):
    print(f"octave {o}:")
    for i, n in enumerate(names):
        print(f"  {n:10s} mean {s[:, o, i].mean():14.0f}  max {s[:, o, i].max():14.0f}")
    t = s[:, o]
    print("  setup cycles/block %.0f  round cycles/round %.0f  rounds/block %.2f  commits/round %.2f  "
          "rect cycles/pt %.0f  total cycles/commit %.0f" % (
              (t[:, 1] / t[:, 5]).mean(), (t[:, 2] / t[:, 6]).mean(), (t[:, 6] / t[:, 5]).mean(),
              (t[:, 8] / t[:, 6]).mean(), (t[:, 3] / np.maximum(t[:, 7], 1)).mean(),
              (t[:, 0] / np.maximum(t[:, 8], 1)).mean()))
    print("  per round: decide %.0f  angles %.0f  verify %.0f  commit %.0f" % tuple(
        (t[:, 9 + k] / t[:, 6]).mean() for k in range(4)))
    print("  seed scan %.0f (%.1f %%, %.0f per 64-pixel chunk)  seed starts %.0f (%.0f per seed)  init %.0f" % (
        t[:, 13].mean(), 100 * (t[:, 13] / t[:, 0]).mean(), t[:, 13].mean() / max(1, names_chunks[o]),
        t[:, 14].mean(), (t[:, 14] / np.maximum(t[:, 4], 1)).mean(), t[:, 15].mean()))
    print("  unaccounted %.1f %%" % (100 * ((t[:, 0] - t[:, 1] - t[:, 2] - t[:, 3] - t[:, 13] - t[:, 14] - t[:, 15])
                                          / t[:, 0]).mean()))
    print("  wave time: mean %.0f  max %.0f cycles" % (t[:, 0].mean(), t[:, 0].max()))
