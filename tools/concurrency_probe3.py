"""Diagnostic for rocprofv3 --kernel-trace: ORB || lines, twice."""
import sys, pathlib
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
for _ in range(2):
    lx.extract_batch(buf.ptr, B, W * H, W)
    orb.extract_batch(buf.ptr, B, W * H, W, (0, 0))
    lib.plvi_device_synchronize()
print("done")
