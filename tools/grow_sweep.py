"""Region-growing stage time vs LDS windows and batch (diagnostic).
usage: python tools/grow_sweep.py "LDS[:RB[:RD]],..." "64,1024" """
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

budgets = (sys.argv[1] if len(sys.argv) > 1 else "6144,6144:2").split(",")
batches = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "64,1024").split(",")]
W, H = 640, 480
allf = synth.device_sequence(max(batches), W, H, 0, "cuda")
for B in batches:
    for bud in budgets:
        parts = bud.split(":")
        os.environ["PLVI_GROW_LDS"] = parts[0]
        os.environ["PLVI_GROW_RB"] = parts[1] if len(parts) > 1 else "64"
        if len(parts) > 2:
            os.environ["PLVI_GROW_RD"] = parts[2]
        else:
            os.environ.pop("PLVI_GROW_RD", None)
        lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
        lx.extract_batch(allf.data_ptr(), B, W * H, W)
        torch.cuda.synchronize()
        lx.profile(True)
        for _ in range(3):
            lx.extract_batch(allf.data_ptr(), B, W * H, W)
        st, runs = lx.profile_read()
        lx.profile(False)
        print(f"B={B} lds={bud} " + " ".join(f"{k}={v / runs:.2f}" for k, v in st.items()), flush=True)
        lx.close()
