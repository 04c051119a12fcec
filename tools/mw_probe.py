"""Region-growing stage time, sequential kernel vs the multi-wave kernel, at
small batches, plus the multi-wave counters (diagnostic).
usage: python tools/mw_probe.py [B,...]"""
import ctypes
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

batches = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,128").split(",")]
W, H = 640, 480
allf = synth.device_sequence(max(batches), W, H, 0, "cuda")
lib = plvi.load()
names = ["disp", "drop", "regrow", "exact", "trivial", "spec_ok", "walk_cyc", "wgrow_cyc", "walks", "blocked",
         "kern_cyc", "spec_cyc", "unused", "blocks", "setup16", "round16"]
# MW_DIAG=1 with a -DPLVI_MW_DIAG=1 variant (PLVI_LIB): 32 counters per task
NS = 32 if os.environ.get("MW_DIAG") == "1" else 16
if NS == 32:
    names += ["w_rg", "w_rg_cyc", "w_first", "w_first_cyc", "inv_d1", "inv_d2", "inv_d3_4", "inv_d5_8", "inv_d9_16",
              "inv_d17p", "chk_lag", "inv_after_reval", "reval_chk", "reval_grow", "wait_n", "wait_ahead"]
for B in batches:
    for mw in (0, 256):
        os.environ["PLVI_GROW_MW"] = str(mw)
        lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B)
        lx.extract_batch(allf.data_ptr(), B, W * H, W)
        torch.cuda.synchronize()
        lx.profile(True)
        for _ in range(5):
            lx.extract_batch(allf.data_ptr(), B, W * H, W)
        st, runs = lx.profile_read()
        lx.profile(False)
        line = f"B={B} mw={mw} " + " ".join(f"{k}={v / runs:.2f}" for k, v in st.items())
        if mw:
            s = torch.zeros(B * 2 * NS, dtype=torch.int32, device="cuda")
            lib.plvi_lines_debug_mw_stats(lx._h, ctypes.c_void_p(s.data_ptr()))
            lx.extract_batch(allf.data_ptr(), B, W * H, W)
            torch.cuda.synchronize()
            lib.plvi_lines_debug_mw_stats(lx._h, ctypes.c_void_p(0))
            a = s.cpu().numpy().reshape(B, 2, NS).mean(axis=0)
            for o in range(2):
                line += f" | oct{o} " + " ".join(f"{n}={a[o, i]:.0f}" for i, n in enumerate(names))
                line += f" setup/blk={16 * a[o, 14] / max(a[o, 13], 1):.0f} round/blk={16 * a[o, 15] / max(a[o, 13], 1):.0f}"
        assert lx.errors() == 0
        print(line, flush=True)
        lx.close()
