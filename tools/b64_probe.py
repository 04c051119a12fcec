"""The bench's batch-64 step (C1/C2 with one batch in flight) for a rocprofv3
kernel trace: warm-up, then a spin_kernel marker, N steps, a marker
(tools/step_timeline.py reads one step's kernel timeline from the trace).
usage: python tools/b64_probe.py [B] [N] [--big [--bigsteps=K]] [--bench-order]"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(argv[0]) if len(argv) > 0 else 64
N = int(argv[1]) if len(argv) > 1 else 10
W, H = 640, 480
big = "--big" in sys.argv  # the bench's situation: 3072-frame handles exist and have run (--bigsteps=K steps)
seq = synth.device_sequence(3072 if big else B, W, H, seed=0, device="cuda:0")
if big:
    ob = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=3072)
    lb = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=3072)
    sb = torch.cuda.Stream()
    nbig = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--bigsteps=")), 3)
    for _ in range(nbig):
        plvi.frame_extract_batch(ob, lb, seq.data_ptr(), 3072, W * H, W, (0, 0), stream=sb.cuda_stream)
    torch.cuda.synchronize()
order = "--bench-order" in sys.argv  # handles created as bench.py does: 2 slots, the drop-in pair, then these
keep = []
if order:
    for _ in range(2):
        keep += [plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=3072),
                 plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=3072), torch.cuda.Stream()]
    keep += [plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H), plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H)]
lib = plvi.load()
o = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
kp, de, co, _, cap = o.outputs()
_, lde, _, lco, lcap = lx.outputs()
i32 = dict(dtype=torch.int32, device="cuda:0")
o4 = [torch.empty((B - 1) * cap, **i32) for _ in range(4)]
lsc = torch.empty(4 * (B - 1) * 2 * lcap, **i32)
lm = torch.empty((B - 1) * lcap, **i32)
lnm = torch.empty(B - 1, **i32)
s = torch.cuda.Stream()
st = s.cuda_stream


def step():
    # as bench.py's batch64 step: the matching issued inside the frame schedule
    plvi.frame_extract_match_batch(o, lx, seq.data_ptr(), B, W * H, W, [x.data_ptr() for x in o4], 0.9,
                                   lsc.data_ptr(), lm.data_ptr(), lnm.data_ptr(), stream=st)


for _ in range(3):
    step()
torch.cuda.synchronize()
torch.cuda._sleep(1000)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    step()
torch.cuda.synchronize()
el = time.perf_counter() - t0
torch.cuda._sleep(1000)
torch.cuda.synchronize()
print(f"B={B}: {el / N * 1e3:.2f} ms per step, {B * N / el:.0f} FPS", flush=True)
assert o.errors() == 0 and lx.errors() == 0
