"""ORB pyramid builders at several batch sizes: average
pyramid time per batch from the extractor's own event pairs (kernel_timing
kind 1: the streaming launch, or the 7 level launches), the whole ORB chain per
batch, and the single-frame drop-in call (plvi_orb_extract, host frame in,
host tables out) -- for PLVI_PYR_LEVELWISE = 0 (always streaming) and the
given thresholds.

usage: python tools/pyr_probe.py [B,B,...] [modes, e.g. 0,256]
"""
import os
import sys
import time
import pathlib

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

Bs = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "1,8,64,256,1024,3072").split(",")]
modes = (sys.argv[2] if len(sys.argv) > 2 else "0,256").split(",")
W, H = 640, 480
seq = synth.device_sequence(max(Bs), W, H, seed=1, device="cuda:0", run=256)
s = torch.cuda.Stream()
for mode in modes:
    os.environ["PLVI_PYR_LEVELWISE"] = mode
    for B in Bs:
        orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B)
        N = 5 if B >= 1024 else 20
        for _ in range(3):
            orb.extract_batch(seq.data_ptr(), B, W * H, W, (0, 0), stream=s.cuda_stream)
        torch.cuda.synchronize()
        orb.kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(N):
            orb.extract_batch(seq.data_ptr(), B, W * H, W, (0, 0), stream=s.cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / N * 1e3
        pt, pn = orb.kernel_timing_read(1)
        bt, bn = orb.kernel_timing_read(0)
        orb.kernel_timing(False)
        assert orb.errors() == 0
        print(f"mode={mode:>5} B={B:5d} pyramid {pt / pn:7.3f} ms  blur+fast {bt / bn:7.3f} ms  "
              f"orb chain {dt:7.3f} ms/batch", flush=True)
        orb.close()
    # single-frame drop-in call
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=1)
    img = synth.frame(3)
    for _ in range(5):
        orb(img)
    ts = []
    for k in range(30):
        t0 = time.perf_counter()
        orb(img)
        ts.append((time.perf_counter() - t0) * 1e3)
    orb.kernel_timing(True)
    orb(img)
    pt, pn = orb.kernel_timing_read(1)
    orb.kernel_timing(False)
    print(f"mode={mode:>5} drop-in plvi_orb_extract median {np.median(ts):.3f} ms p90 {np.percentile(ts, 90):.3f}"
          f"  (pyramid {pt / max(pn, 1):.3f} ms)", flush=True)
    orb.close()
