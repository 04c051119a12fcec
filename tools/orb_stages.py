"""ORB extractor alone: per-stage times (HIP events, plvi profile) and the
ORB-only rate at batch B.  usage: python tools/orb_stages.py [B] [N]"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W, H = 640, 480
seq = synth.device_sequence(B, W, H, seed=0, device="cuda:0")
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
s = torch.cuda.Stream()
st = s.cuda_stream
orb.extract_batch(seq.data_ptr(), B, W * H, W, (0, 0), stream=st)
torch.cuda.synchronize()
orb.profile(True)
for _ in range(N):
    orb.extract_batch(seq.data_ptr(), B, W * H, W, (0, 0), stream=st)
torch.cuda.synchronize()
stg, runs = orb.profile_read()
orb.profile(False)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(N):
    orb.extract_batch(seq.data_ptr(), B, W * H, W, (0, 0), stream=st)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / N
print(f"B={B} orb-only {ms:.2f} ms ({B / ms * 1e3:.0f} FPS) | " +
      " ".join(f"{k}={v / runs:.2f}" for k, v in stg.items()), flush=True)
assert orb.errors(st) == 0
