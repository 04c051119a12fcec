"""Diagnostic: capture a plvi step into a HIP graph and replay it.
usage: python tools/graph_probe.py {knn|orb|lines|frame}"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

what = sys.argv[1]
n = 16
seq = synth.device_sequence(n, 640, 480, seed=5, device="cuda:0")
torch.cuda.synchronize()
lib = plvi.load()
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=n)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=n)
kp, de, co, _, cap = orb.outputs()
outs = [torch.empty(((n - 1) * cap,), dtype=torch.int32, device="cuda:0") for _ in range(4)]
s = torch.cuda.Stream()


def step(st):
    if what in ("orb",):
        orb.extract_batch(seq.data_ptr(), n, 640 * 480, 640, stream=st)
    if what in ("lines",):
        lx.extract_batch(seq.data_ptr(), n, 640 * 480, 640, stream=st)
    if what in ("frame",):
        plvi.frame_extract_batch(orb, lx, seq.data_ptr(), n, 640 * 480, 640, stream=st)
    if what in ("knn", "frame"):
        assert lib.plvi_hamming_knn2_batch(de + cap * 32, co + 4, cap, de, co, cap, n - 1,
                                           *[o.data_ptr() for o in outs], st) == 0


step(s.cuda_stream)
torch.cuda.synchronize()
print(what, "direct ok", flush=True)
g = plvi.StepGraph(step, s.cuda_stream)
print(what, "captured", flush=True)
g.launch()
torch.cuda.synchronize()
print(what, "replayed ok", flush=True)
