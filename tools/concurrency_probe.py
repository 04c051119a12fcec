"""Diagnostic: do the ORB and line extractors overlap on two streams?"""
import sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch
import plvi
from plvi import synth

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
W, H = 640, 480
frames = torch.from_numpy(synth.batch(B, W, H)).cuda()
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
lib = plvi.load()
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, n=3):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


o = lambda s=None: orb.extract_batch(frames.data_ptr(), B, W * H, W, (0, 0), stream=s)
l = lambda s=None: lx.extract_batch(frames.data_ptr(), B, W * H, W, stream=s)
print("orb torch-stream   %.2f ms" % t(lambda: o(sA.cuda_stream)))
print("lines torch-stream %.2f ms" % t(lambda: l(sB.cuda_stream)))
print("both torch-streams %.2f ms" % t(lambda: (l(sB.cuda_stream), o(sA.cuda_stream))))
print("orb own-stream     %.2f ms" % t(lambda: (o(), lib.plvi_device_synchronize())))
print("lines own-stream   %.2f ms" % t(lambda: (l(), lib.plvi_device_synchronize())))
print("both own-streams   %.2f ms" % t(lambda: (l(), o(), lib.plvi_device_synchronize())))
