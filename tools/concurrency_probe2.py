"""Diagnostic without torch: ORB || lines on the handles' own streams."""
import sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi
from plvi import synth

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
W, H = 640, 480
fr = synth.batch(B, W, H)
buf = plvi.DeviceBuffer(fr.nbytes); buf.upload(fr)
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
lib = plvi.load()


def t(fn, n=3):
    fn(); lib.plvi_device_synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    lib.plvi_device_synchronize()
    return (time.perf_counter() - t0) / n * 1e3


o = lambda: orb.extract_batch(buf.ptr, B, W * H, W, (0, 0))
l = lambda: lx.extract_batch(buf.ptr, B, W * H, W)
print("orb   %.2f ms" % t(o))
print("lines %.2f ms" % t(l))
print("both  %.2f ms" % t(lambda: (l(), o())))
print("both (orb first) %.2f ms" % t(lambda: (o(), l())))
