"""SURVEY §8c diagnostic: how often does the reference's allocator-dependent
octree tie-break (DistributeOctTree sorts (size, ExtractorNode*) pairs,
ORBextractor.cc:679-683) change the extracted keypoints?

Runs the oracle ORB extractor on N frames with three tie orders for
equal-size nodes — creation order (a bump allocator; the canonical rule the
HIP path and the parity tests use), reverse creation order, and a
pseudo-random order (malloc reusing freed list nodes) — and reports the
fraction of (frame, level) pairs and of frames whose keypoint sets differ
from the canonical one.  usage: python tools/octree_tie_diag.py [N]"""
import ctypes
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import oracle_lib  # noqa: E402
from plvi import synth  # noqa: E402
from util import real_frames  # noqa: E402


def run(n_synth=16):
    lib = oracle_lib.load()
    lib.oracle_orb_set_tie_mode.argtypes = [ctypes.c_int]
    frames = [synth.frame(500 + i) for i in range(n_synth)]
    fr = real_frames()
    frames += [fr[k] for k in sorted(fr)]
    out = {}
    base = []
    for mode in (0, 1, 2):
        lib.oracle_orb_set_tie_mode(mode)
        res = [oracle_lib.orb_extract(f)[1] for f in frames]
        if mode == 0:
            base = res
            continue
        lv_diff = lv_tot = fr_diff = 0
        sym = kept = 0
        for a, b in zip(base, res):
            diff_any = False
            for l in range(8):
                sa = set(zip(a["x"][a["octave"] == l].tolist(), a["y"][a["octave"] == l].tolist()))
                sb = set(zip(b["x"][b["octave"] == l].tolist(), b["y"][b["octave"] == l].tolist()))
                lv_tot += 1
                sym += len(sa ^ sb)
                kept += len(sa)
                if sa != sb:
                    lv_diff += 1
                    diff_any = True
            fr_diff += diff_any
        out[{1: "reverse", 2: "random"}[mode]] = (lv_diff / lv_tot, fr_diff / len(frames), sym / (2 * kept))
    lib.oracle_orb_set_tie_mode(0)
    return len(frames), out


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    nf, out = run(n)
    for k, (lv, fr_, kp) in out.items():
        print(f"{k:8s}: {100 * lv:5.1f} % of (frame, level) pairs and {100 * fr_:5.1f} % of {nf} frames differ; "
              f"{100 * kp:4.2f} % of keypoints replaced")
