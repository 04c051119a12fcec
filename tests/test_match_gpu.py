"""Hamming matchers: HIP kNN-2 / LineMatcher vs the CPU oracle (BFMatcher
tie rules), including planted ties and duplicate rows."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from util import near_duplicate_descriptors

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nq,nt", [(1, 2), (7, 5), (200, 200), (1000, 1000), (300, 1500)])
def test_knn2_matches_oracle(plvi_lib, nq, nt):
    rng = np.random.default_rng(nq * 7 + nt)
    q, t = near_duplicate_descriptors(rng, nt, nq)
    got = plvi.hamming_knn2(q, t)
    exp = ol.knn2(q, t)
    for g, e, name in zip(got, exp, ["idx0", "d0", "idx1", "d1"]):
        assert np.array_equal(g, e), name


def test_knn2_ties_keep_lower_index(plvi_lib):
    rng = np.random.default_rng(5)
    t = rng.integers(0, 256, size=(64, 32), dtype=np.uint8)
    t[10] = t[3]; t[40] = t[3]; t[41] = t[7]
    q = t[[3, 7, 10, 41]].copy()
    got = plvi.hamming_knn2(q, t)
    exp = ol.knn2(q, t)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    assert got[0][0] == 3 and got[2][0] == 10 and got[1][0] == 0 and got[3][0] == 0


def test_line_match_nnr_and_mutual(plvi_lib):
    rng = np.random.default_rng(9)
    q, t = near_duplicate_descriptors(rng, 180, 200, p_flip=0.05)
    for nnr in (0.9, 0.75):
        assert plvi.LineMatcher.matchNNR(q, t, nnr)[0] == ol.match_nnr(q, t, nnr)[0]
        assert np.array_equal(plvi.LineMatcher.matchNNR(q, t, nnr)[1], ol.match_nnr(q, t, nnr)[1])
        n, m = plvi.LineMatcher.match(q, t, nnr)
        ne, me = ol.match(q, t, nnr)
        assert n == ne and np.array_equal(m, me)
