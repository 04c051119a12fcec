"""Capture a plvi step into a HIP graph (plvi_graph_*), replay it and compare
every output table with the step issued call by call.
usage: python tools/graph_probe.py {knn|orb|lines|frame} [n_frames]
Prints "<what> replay equal" and exits 0 when the replay reproduces the
direct step bit for bit (tests/test_frame_gpu.py runs it as a child process,
so a crash inside the runtime fails one test, not the suite)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

what = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
seq = synth.device_sequence(n, 640, 480, seed=5, device="cuda:0")
torch.cuda.synchronize()
lib = plvi.load()
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=n)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=n)
kp, de, co, _, cap = orb.outputs()
kl, lde, lfn, lco, lcap = lx.outputs()
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


def tables():
    torch.cuda.synchronize()
    t = [plvi.download(p, np.zeros(b, np.uint8)) for p, b in
         ((co, 4 * n), (kp, 28 * cap * n), (de, 32 * cap * n), (lco, 4 * n), (kl, 68 * lcap * n),
          (lde, 32 * lcap * n), (lfn, 24 * lcap * n))]
    return t + [o.cpu().numpy().copy() for o in outs]


def clear():
    torch.cuda.synchronize()
    for p, b in ((co, 4 * n), (kp, 28 * cap * n), (de, 32 * cap * n), (lco, 4 * n), (kl, 68 * lcap * n),
                 (lde, 32 * lcap * n), (lfn, 24 * lcap * n)):
        junk = np.full(b, 0xA5, np.uint8)
        assert lib.plvi_memcpy(p, junk.ctypes.data, b, 1) == 0
    for o in outs:
        o.fill_(-7)
    torch.cuda.synchronize()


step(s.cuda_stream)
ref = tables()
hip = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})
print(what, n, "direct ok; HIP runtime", hip, flush=True)
clear()
g = plvi.StepGraph(step, s.cuda_stream)
print(what, "captured", flush=True)
g.launch()
got = tables()
print(what, "replayed", flush=True)
bad = [i for i, (a, b) in enumerate(zip(ref, got)) if not np.array_equal(a, b)]
clear()
g.launch()
g.launch()
got2 = tables()
bad += [i for i, (a, b) in enumerate(zip(ref, got2)) if not np.array_equal(a, b)]
assert orb.errors() == 0 and lx.errors() == 0
if bad:
    print(what, "replay differs in tables", sorted(set(bad)), flush=True)
    sys.exit(1)
print(what, "replay equal", flush=True)
