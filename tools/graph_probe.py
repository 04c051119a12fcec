"""Capture a plvi step into a HIP graph (plvi_graph_*), replay it and compare
every output table with the step issued call by call.
usage: python tools/graph_probe.py {knn|orb|lines|frame} [n_frames] [--torch]
Without --torch the process never imports torch, so the library runs on the
system ROCm runtime (/opt/rocm); with --torch, torch is imported first and
its bundled HIP runtime is the one mapped (the frame schedule's capture is
then refused with PLVI_E_CAPTURE on runtimes < 7.2).  Prints
"<what> replay equal" (or "<what> capture refused") and exits 0 on success;
tests/test_frame_gpu.py runs it as a child process, so a crash inside the
runtime fails one test, not the suite."""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
use_torch = "--torch" in sys.argv
args = [a for a in sys.argv[1:] if a != "--torch"]
if use_torch:
    import torch  # noqa: F401,E402
else:
    import os
    os.environ["PLVI_NO_TORCH"] = "1"  # plvi.load() would import torch (and its HIP runtime) first
import numpy as np  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

what = args[0]
n = int(args[1]) if len(args) > 1 else 16
W, H = 640, 480
lib = plvi.load()
frames = synth.batch(n, W, H, seed0=5)
fb = plvi.DeviceBuffer(frames.nbytes)
fb.upload(frames)
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=n)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=n)
kp, de, co, _, cap = orb.outputs()
kl, lde, lfn, lco, lcap = lx.outputs()
outs = [plvi.DeviceBuffer(4 * (n - 1) * cap) for _ in range(4)]
sp = ctypes.c_void_p()
assert lib.plvi_stream_create(ctypes.byref(sp)) == 0
stream = sp.value


def step(st):
    if what in ("orb",):
        orb.extract_batch(fb.ptr, n, W * H, W, stream=st)
    if what in ("lines",):
        lx.extract_batch(fb.ptr, n, W * H, W, stream=st)
    if what in ("frame",):
        plvi.frame_extract_batch(orb, lx, fb.ptr, n, W * H, W, stream=st)
    if what in ("knn", "frame"):
        assert lib.plvi_hamming_knn2_batch(de + cap * 32, co + 4, cap, de, co, cap, n - 1,
                                           *[o.ptr for o in outs], st) == 0


TABLES = ((co, 4 * n), (kp, 28 * cap * n), (de, 32 * cap * n), (lco, 4 * n), (kl, 68 * lcap * n),
          (lde, 32 * lcap * n), (lfn, 24 * lcap * n))


def tables():
    """The valid part of every table: the first count rows of each frame
    (pair) slot; rows beyond a frame's count are not outputs."""
    assert lib.plvi_stream_synchronize(stream) == 0
    t = [plvi.download(p, np.zeros(b, np.uint8)) for p, b in TABLES]
    cnt, lcnt = t[0].view(np.int32), t[3].view(np.int32)
    out = [t[0], t[3]]
    for tab, c, cp, row in ((t[1], cnt, cap, 28), (t[2], cnt, cap, 32), (t[4], lcnt, lcap, 68),
                            (t[5], lcnt, lcap, 32), (t[6], lcnt, lcap, 24)):
        out.append(np.concatenate([tab[f * cp * row:(f * cp + c[f]) * row] for f in range(n)]))
    for o in outs:
        v = o.download(np.zeros(o.nbytes, np.uint8)).view(np.int32)
        out.append(np.concatenate([v[p * cap:p * cap + cnt[p + 1]] for p in range(n - 1)]) if what in ("knn", "frame")
                   else v)
    return out


def clear():
    assert lib.plvi_stream_synchronize(stream) == 0
    for p, b in TABLES + tuple((o.ptr, o.nbytes) for o in outs):
        junk = np.full(b, 0xA5, np.uint8)
        assert lib.plvi_memcpy(p, junk.ctypes.data, b, 1) == 0


step(stream)
ref = tables()
hip = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln})
ver = ctypes.c_int()
ctypes.CDLL(hip[0]).hipRuntimeGetVersion(ctypes.byref(ver))
print(what, n, "direct ok; HIP runtime", hip, ver.value, flush=True)
clear()
try:
    g = plvi.StepGraph(step, stream)
except plvi.PlviError as e:
    if e.code == plvi.PLVI_E_CAPTURE:
        print(what, "capture refused (PLVI_E_CAPTURE, runtime", ver.value, ")", flush=True)
        sys.exit(0 if ver.value < 70200000 else 1)
    raise
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
