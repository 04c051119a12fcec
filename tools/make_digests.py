"""tests/golden/oracle_digests.json: SHA-256 of the CPU oracle's outputs on
the reference's 10 real frames (tests/golden/frames.npz), so that any change
of the oracle's behaviour shows up in tests/test_golden_digests.py.

Per frame: ORB (monoIndex, keypoints in cv::KeyPoint layout, descriptors)
for ORBextractor(1000, 1.2, 8, 20, 7), lines (KeyLines, LBD descriptors,
line functions) for Lineextractor(200, 0, 0.8, 2, 2.0); per consecutive
pair of the same camera: ORB kNN-2 and LineMatcher::match (ratio 0.9).
Also the counts, for a readable diff.  Run: python tools/make_digests.py
"""
import hashlib
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))


def h(*arrays):
    d = hashlib.sha256()
    for a in arrays:
        d.update(memoryview(a).tobytes() if hasattr(a, "tobytes") else str(a).encode())
    return d.hexdigest()


def digests():
    import numpy as np
    import oracle_lib as ol
    from util import real_frames
    fr = real_frames()
    out = {}
    ext = {}
    for k in sorted(fr):
        m, kp, de = ol.orb_extract(fr[k])
        kl, ld, fn = ol.line_extract(fr[k])
        ext[k] = (de, ld)
        out[k] = {"orb_n": int(len(kp)), "orb_mono": int(m), "orb": h(np.int32(m), kp, de),
                  "lines_n": int(len(kl)), "lines": h(kl, ld, fn)}
    for cam, n in (("euroc", 5), ("rgb", 5)):
        for i in range(1, n):
            a = f"{cam}{i}" if cam == "euroc" else f"rgb{i}_gray"
            b = f"{cam}{i + 1}" if cam == "euroc" else f"rgb{i + 1}_gray"
            knn = ol.knn2(ext[b][0], ext[a][0])
            nm, m12 = ol.match(ext[b][1], ext[a][1], 0.9)
            out[f"{b}->{a}"] = {"knn2": h(*knn), "lmatch_n": int(nm), "lmatch": h(m12)}
    return out


if __name__ == "__main__":
    p = ROOT / "tests" / "golden" / "oracle_digests.json"
    p.write_text(json.dumps(digests(), indent=1, sort_keys=True) + "\n")
    print(p)
