"""The CPU oracle pinned to its committed outputs on the reference's 10 real
frames (tests/golden/oracle_digests.json, tools/make_digests.py): any change
of the oracle's behaviour must show up here and be re-committed on purpose.
The GPU half runs the product on the same frames and pairs and compares it
with the oracle, bit for bit (the real euroc1 <-> euroc2 ... pairs are
matched with ORB kNN-2 and LineMatcher::match)."""
import json
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

GOLD = json.loads((ROOT / "tests" / "golden" / "oracle_digests.json").read_text())


def test_oracle_outputs_match_committed_digests():
    import make_digests
    got = make_digests.digests()
    assert set(got) == set(GOLD)
    bad = [k for k in GOLD if got[k] != GOLD[k]]
    assert not bad, {k: (got[k], GOLD[k]) for k in bad[:3]}


@pytest.mark.gpu
def test_real_frames_and_pairs_gpu_equal_oracle(plvi_lib):
    import oracle_lib as ol
    import plvi
    from util import real_frames
    fr = real_frames()
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480)
    outs = {}
    for k in sorted(fr):
        m, kp, de = orb(fr[k])
        kl, ld, fn = lx(fr[k])
        em, ek, ed = ol.orb_extract(fr[k])
        assert m == em and kp.tobytes() == ek.tobytes() and np.array_equal(de, ed), k
        ekl, eld, efn = ol.line_extract(fr[k])
        assert kl.tobytes() == ekl.tobytes() and np.array_equal(ld, eld) and fn.tobytes() == efn.tobytes(), k
        assert GOLD[k]["orb_n"] == len(kp) and GOLD[k]["lines_n"] == len(kl)
        outs[k] = (de, ld)
    for i in range(1, 5):
        for a, b in ((f"euroc{i}", f"euroc{i + 1}"), (f"rgb{i}_gray", f"rgb{i + 1}_gray")):
            got = plvi.hamming_knn2(outs[b][0], outs[a][0])
            exp = ol.knn2(outs[b][0], outs[a][0])
            assert all(np.array_equal(g, e) for g, e in zip(got, exp)), (a, b)
            ng, mg = plvi.LineMatcher.match(outs[b][1], outs[a][1], 0.9)
            ne, me = ol.match(outs[b][1], outs[a][1], 0.9)
            assert ng == ne == GOLD[f"{b}->{a}"]["lmatch_n"] and np.array_equal(mg, me), (a, b)
