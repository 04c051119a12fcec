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


def test_line_match_batch_device(plvi_lib):
    rng = np.random.default_rng(21)
    P, cap = 5, 64
    d1 = np.zeros((P, cap, 32), np.uint8)
    d2 = np.zeros((P, cap, 32), np.uint8)
    n1 = np.array([64, 10, 2, 1, 40], np.int32)
    n2 = np.array([60, 12, 5, 30, 0], np.int32)
    for p in range(P):
        q, t = near_duplicate_descriptors(rng, max(n2[p], 1), max(n1[p], 1), p_flip=0.05)
        d1[p, :n1[p]] = q[:n1[p]]
        d2[p, :n2[p]] = t[:n2[p]]
    bufs = {k: plvi.DeviceBuffer(v.nbytes) for k, v in dict(d1=d1, d2=d2, n1=n1, n2=n2).items()}
    for k, v in dict(d1=d1, d2=d2, n1=n1, n2=n2).items():
        bufs[k].upload(v)
    scratch = plvi.DeviceBuffer(4 * P * 2 * cap * 4)
    m12 = plvi.DeviceBuffer(P * cap * 4)
    nm = plvi.DeviceBuffer(P * 4)
    rc = plvi.load().plvi_line_match_batch(bufs["d1"].ptr, bufs["n1"].ptr, cap, bufs["d2"].ptr, bufs["n2"].ptr, cap, P,
                                           0.9, scratch.ptr, m12.ptr, nm.ptr, None)
    assert rc == 0
    plvi.load().plvi_device_synchronize()
    got = m12.download(np.zeros((P, cap), np.int32))
    cnt = nm.download(np.zeros(P, np.int32))
    for p in range(P):
        if n1[p] >= 2 and n2[p] >= 2:
            ne, me = ol.match(d1[p, :n1[p]], d2[p, :n2[p]], 0.9)
            assert cnt[p] == ne and np.array_equal(got[p, :n1[p]], me)
        else:
            assert cnt[p] == 0


@pytest.mark.parametrize("nq,nt", [(0, 5), (4, 0), (6, 1)])
def test_knn2_degenerate_sizes(plvi_lib, nq, nt):
    # knnMatch with fewer than 2 train rows leaves the missing neighbours at
    # (-1, INT_MAX) in the oracle's BFMatcher restatement; nq == 0 is a no-op
    rng = np.random.default_rng(100 + nq * 3 + nt)
    q = rng.integers(0, 256, size=(nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(nt, 32), dtype=np.uint8)
    got = plvi.hamming_knn2(q, t)
    exp = ol.knn2(q, t)
    for g, e, name in zip(got, exp, ["idx0", "d0", "idx1", "d1"]):
        assert g.shape == (nq,) and np.array_equal(g, e), name


def test_knn2_all_equal_targets_and_max_distance(plvi_lib):
    # every train row identical: all distances tie, first two indices win;
    # query = bitwise complement of the train rows: distance 256 everywhere
    rng = np.random.default_rng(77)
    row = rng.integers(0, 256, size=32, dtype=np.uint8)
    t = np.tile(row, (300, 1))
    q = np.stack([row, ~row, row ^ 1])  # row ^ 1 flips one bit per byte
    got = plvi.hamming_knn2(q, t)
    exp = ol.knn2(q, t)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)
    assert list(got[0]) == [0, 0, 0] and list(got[2]) == [1, 1, 1]
    assert list(got[1]) == [0, 256, 32] and list(got[3]) == [0, 256, 32]


def test_line_match_nnr_rejects_single_train_row(plvi_lib):
    # LineMatcher::matchNNR reads matches_[idx][1] (LineMatcher.cpp:41-61),
    # undefined with one train row: the C-ABI refuses instead of guessing
    rng = np.random.default_rng(3)
    q = rng.integers(0, 256, size=(4, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(1, 32), dtype=np.uint8)
    with pytest.raises(plvi.PlviError):
        plvi.LineMatcher.matchNNR(q, t, 0.9)
