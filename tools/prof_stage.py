"""Drive one stage family on a device-resident batch for PMC / kernel-trace
profiling (diagnostic): python tools/prof_stage.py {orb|lines|frame} [B] [reps]."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "orb"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
W, H = 640, 480
frames = torch.from_numpy(synth.batch(B, W, H, seed0=0)).cuda()
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
s = torch.cuda.Stream()
for _ in range(reps):
    if what in ("orb", "frame"):
        if what == "orb":
            orb.extract_batch(frames.data_ptr(), B, W * H, W, stream=s.cuda_stream)
        else:
            plvi.frame_extract_batch(orb, lx, frames.data_ptr(), B, W * H, W, stream=s.cuda_stream)
    if what == "lines":
        lx.extract_batch(frames.data_ptr(), B, W * H, W, stream=s.cuda_stream)
    torch.cuda.synchronize()
print("done", what, B, reps)
