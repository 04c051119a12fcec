"""PMC target (diagnostic): the calibration kernels of tools/calib/pmc_calib.hip
on 1 GiB buffers (4x the 256 MiB Infinity Cache, so every byte streams from
HBM), then the frame schedule (plvi_frame_extract_batch) on B frames, R times.
usage: python tools/pmc_frame.py [B] [R]"""
import ctypes
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
CAL_BYTES = 1 << 30
cal = ctypes.CDLL(str(ROOT / "tools" / "lib" / "libplvi_calib.so"))
cal.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
src = torch.randint(0, 255, (CAL_BYTES,), dtype=torch.uint8, device="cuda")
dst = torch.empty(CAL_BYTES, dtype=torch.uint8, device="cuda")
for mode in range(5):
    assert cal.calib_run(mode, src.data_ptr(), dst.data_ptr(), CAL_BYTES, None) == 0
torch.cuda.synchronize()
del src, dst
W, H = 640, 480
seq = synth.device_sequence(B, W, H, seed=1, device="cuda:0")
orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
s = torch.cuda.Stream()
for _ in range(R):
    plvi.frame_extract_batch(orb, lx, seq.data_ptr(), B, W * H, W, (0, 0), stream=s.cuda_stream)
torch.cuda.synchronize()
print("ok", orb.errors(), lx.errors(), "calib_bytes", CAL_BYTES, "batch", B, "reps", R)
