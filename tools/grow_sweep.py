"""Region-growing stage time vs LDS window budget and batch (diagnostic).
usage: python tools/grow_sweep.py "12288,40960,81920" "64,1024" """
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

budgets = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "12288,40960").split(",")]
batches = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "64,1024").split(",")]
W, H = 640, 480
allf = torch.from_numpy(synth.batch(max(batches), W, H, seed0=0)).cuda()
for B in batches:
    for bud in budgets:
        os.environ["PLVI_GROW_LDS"] = str(bud)
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
