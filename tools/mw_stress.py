"""Diagnostic: repeatability of the multi-wave region growing.  The same
batch is extracted REPS times; every run's keylines / LBD descriptors are
compared with the first run's and with the sequential kernel's
(PLVI_GROW_MW=0).  Prints the number of differing frames per run.
usage: python tools/mw_stress.py [n_frames] [reps]"""
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import torch  # noqa: E402

import plvi  # noqa: E402
from plvi import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
seq = synth.device_sequence(n, 640, 480, seed=5, device="cuda:0")
torch.cuda.synchronize()


def run(lx):
    lx.extract_batch(seq.data_ptr(), n, 640 * 480, 640)
    torch.cuda.synchronize()
    assert lx.errors() == 0
    kl, de, fn, co, cap = lx.outputs()
    cnt = plvi.download(co, np.zeros(n, np.int32))
    k = plvi.download(kl, np.zeros(n * cap, plvi.KEYLINE_DTYPE))
    return [k[f * cap:f * cap + cnt[f]].tobytes() for f in range(n)]


os.environ["PLVI_GROW_MW"] = "0"
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=n)
seqref = run(lx)
lx.close()
os.environ["PLVI_GROW_MW"] = "256"
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=n)
first = run(lx)
bad_seq = [f for f in range(n) if first[f] != seqref[f]]
tot = len(bad_seq)
print(f"run 0: frames != sequential {bad_seq}", flush=True)
for r in range(1, reps):
    out = run(lx)
    d0 = [f for f in range(n) if out[f] != first[f]]
    ds = [f for f in range(n) if out[f] != seqref[f]]
    tot += len(ds)
    print(f"run {r}: != run0 {d0}  != sequential {ds}", flush=True)
print(f"total frame mismatches vs sequential over {reps} runs: {tot}")
