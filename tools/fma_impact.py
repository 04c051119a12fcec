"""How much the reference build's FMA contraction changes the path's outputs.

The reference's own code is compiled by GCC 9.4 at -O3 -march=native, which
fuses the multiply-adds tests/test_ref_objects.py lists (oracle/ref_fma.h).
This builds the oracle a second time with -DORACLE_NO_REF_FMA (every site
unfused, the assumption of rounds 1-4) and counts, on the reference's real
frames and on synthetic ones, the outputs that differ between the two:
ORB keypoints / descriptor bytes, keylines, LBD descriptors, line functions.

Run: python tools/fma_impact.py [n_synth]   (CPU only; a few minutes)
"""
import json
import os
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent


def dump(out, n_synth):
    sys.path.insert(0, str(ROOT / "tests"))
    sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
    import oracle_lib as ol
    from plvi import synth
    from util import real_frames
    fr = real_frames()
    imgs = [fr[k] for k in sorted(fr)] + list(synth.batch(n_synth, seed0=4242))
    res = {}
    for i, img in enumerate(imgs):
        _, kp, de = ol.orb_extract(img)
        kl, ld, fn = ol.line_extract(img)
        res[f"kp{i}"], res[f"de{i}"], res[f"kl{i}"], res[f"ld{i}"], res[f"fn{i}"] = kp, de, kl, ld, fn
    np.savez(out, n=len(imgs), **res)


def main():
    n_synth = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    if len(sys.argv) > 2 and sys.argv[2] == "--dump":
        dump(sys.argv[3], n_synth)
        return
    with tempfile.TemporaryDirectory() as td:
        nofma = os.path.join(td, "liboracle_nofma.so")
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), f"OUT={nofma}", "EXTRA=-DORACLE_NO_REF_FMA"],
                       check=True)
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
        outs = {}
        for tag, lib in (("fma", None), ("nofma", nofma)):
            env = dict(os.environ)
            env.pop("ORACLE_LIB", None)
            if lib:
                env["ORACLE_LIB"] = lib
            outs[tag] = os.path.join(td, tag + ".npz")
            subprocess.run([sys.executable, __file__, str(n_synth), "--dump", outs[tag]], check=True, env=env)
        a, b = np.load(outs["fma"]), np.load(outs["nofma"])
        n = int(a["n"])
        tot = {"frames": n, "frames_any_diff": 0, "orb_frames_diff": 0, "orb_kp_diff": 0, "orb_desc_bytes_diff": 0,
               "orb_desc_rows_diff": 0, "orb_kps": 0, "line_frames_diff": 0, "keylines_diff": 0,
               "keyline_count_diff": 0, "lbd_rows_diff": 0, "linefn_diff": 0, "keylines": 0}
        for i in range(n):
            kpa, kpb, dea, deb = a[f"kp{i}"], b[f"kp{i}"], a[f"de{i}"], b[f"de{i}"]
            tot["orb_kps"] += len(kpa)
            any_ = False
            if len(kpa) != len(kpb) or kpa.tobytes() != kpb.tobytes() or dea.tobytes() != deb.tobytes():
                tot["orb_frames_diff"] += 1
                any_ = True
                if len(kpa) == len(kpb):
                    tot["orb_kp_diff"] += int((kpa != kpb).sum())
                    tot["orb_desc_bytes_diff"] += int((dea != deb).sum())
                    tot["orb_desc_rows_diff"] += int((dea != deb).any(1).sum())
            kla, klb = a[f"kl{i}"], b[f"kl{i}"]
            tot["keylines"] += len(kla)
            if len(kla) != len(klb):
                tot["keyline_count_diff"] += 1
                tot["line_frames_diff"] += 1
                any_ = True
            elif kla.tobytes() != klb.tobytes() or a[f"ld{i}"].tobytes() != b[f"ld{i}"].tobytes() or \
                    a[f"fn{i}"].tobytes() != b[f"fn{i}"].tobytes():
                tot["line_frames_diff"] += 1
                any_ = True
                tot["keylines_diff"] += int((kla != klb).sum())
                tot["lbd_rows_diff"] += int((a[f"ld{i}"] != b[f"ld{i}"]).any(1).sum())
                tot["linefn_diff"] += int((a[f"fn{i}"] != b[f"fn{i}"]).any(-1).sum()) if a[f"fn{i}"].ndim > 1 else \
                    int((a[f"fn{i}"] != b[f"fn{i}"]).sum())
            tot["frames_any_diff"] += any_
        print(json.dumps(tot, indent=1))


if __name__ == "__main__":
    main()
