"""Micro run of the line extractor alone (rocprofv3 target): B frames, N batches."""
import sys
import pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W, H = 640, 480
seq = synth.device_sequence(B, W, H, seed=1, device="cuda:0", run=256)
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
s = torch.cuda.Stream()
for _ in range(N):
    lx.extract_batch(seq.data_ptr(), B, W * H, W, stream=s.cuda_stream)
torch.cuda.synchronize()
print("ok", lx.errors())
