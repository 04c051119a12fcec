"""ORBmatcher::SearchByBoW (src/ORBmatcher.cc:269-471) and the descriptor
distances (ORBmatcher.cc:2350-2366, LineMatcher.cpp:487-499).

Parity unpinned: the reference has no tests for SearchByBoW;
the oracle restates the cited lines and is checked here on hand-built known
answers, then the HIP kernel is compared with it on synthetic FeatureVectors.

Two-camera Frames (F.Nleft != -1, ORBmatcher.cc:321-420): the right-image
ratio test is `... || true` (ORBmatcher.cc:405), i.e. every right best match
within TH_LOW is kept; the oracle (match_oracle.cpp) and the kernel (bow.hip)
both encode that (test_oracle_search_by_bow_two_cameras_known_answers)."""
import numpy as np
import pytest

import oracle_lib
import util


def _desc(rng, n):
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


def _flip(d, nbits, rng):
    bits = np.unpackbits(d.copy())
    idx = rng.choice(256, nbits, replace=False)
    bits[idx] ^= 1
    return np.packbits(bits)


def test_oracle_search_by_bow_known_answers():
    rng = np.random.default_rng(5)
    kf = _desc(rng, 4)
    f = np.stack([_flip(kf[0], 10, rng), _flip(kf[0], 12, rng), _flip(kf[1], 60, rng), _flip(kf[2], 5, rng),
                  _flip(kf[3], 3, rng)])
    kf_angle = np.array([10, 20, 30, 40], np.float32)
    f_angle = np.array([0, 0, 0, 25, 30], np.float32)
    live = np.array([1, 1, 1, 0], np.uint8)
    kf_fv = {7: [0, 1], 9: [2, 3]}
    f_fv = {7: [0, 1, 2], 9: [3, 4], 11: []}
    n, m = oracle_lib.search_by_bow(kf, kf_angle, live, kf_fv, f, f_angle, f_fv, 0.9, check_orientation=False)
    # KF0 -> F0 (10 bits) passes 10 < 0.9*12; KF1 only has F2 at ~60 bits left (> TH_LOW 50): no match.
    # KF2 -> F3 (5 bits) vs F4 (~3 + 2*...): F3 is the best; KF3 is not live.
    assert m[0] == 0 and m[1] == -1 and m[2] == -1 and m[3] == 2 and m[4] == -1
    assert n == 2
    # orientation: rotations 10 and 5 degrees both fall in bin 0 -> both kept
    n2, m2 = oracle_lib.search_by_bow(kf, kf_angle, live, kf_fv, f, f_angle, f_fv, 0.9, check_orientation=True)
    assert n2 == 2 and (m2 == m).all()


def test_oracle_search_by_bow_two_cameras_known_answers():
    """The two-camera branch (ORBmatcher.cc:321-420, F.Nleft != -1): a best / second pair per camera; the right
    best is taken without a ratio test, but only inside the left best's TH_LOW test."""
    rng = np.random.default_rng(9)
    kf = _desc(rng, 3)
    # F: left keypoints 0..2, right keypoints 3..5 (Nleft = 3)
    f = np.stack([_flip(kf[0], 10, rng), _flip(kf[0], 11, rng), _flip(kf[1], 8, rng),    # left
                  _flip(kf[0], 20, rng), _flip(kf[1], 90, rng), _flip(kf[2], 4, rng)])   # right
    kf_angle = np.zeros(3, np.float32)
    f_angle = np.zeros(6, np.float32)
    live = np.ones(3, np.uint8)
    kf_fv = {5: [0, 1, 2]}
    f_fv = {5: [0, 1, 2, 3, 4, 5]}
    n, m = oracle_lib.search_by_bow(kf, kf_angle, live, kf_fv, f, f_angle, f_fv, 0.75, check_orientation=False,
                                    f_nleft=3)
    # KF0: left best F0 (10) fails the ratio vs F1 (11), yet its right best F3 (20 <= 50) is taken (`|| true`).
    # KF1: left best F2 (8) passes; its right side holds only F4 (~90 > TH_LOW): left only.
    # KF2: no left candidate within TH_LOW (F1 ~ random vs KF2) -> its right best F5 (4 bits) is NOT taken.
    assert list(m) == [-1, -1, 1, 0, -1, -1]
    assert n == 2
    # one camera (Nleft = -1): all six compete; KF0 -> F0 (10 < 0.75 * 11 fails) ... the same rule as before
    n1, m1 = oracle_lib.search_by_bow(kf, kf_angle, live, kf_fv, f, f_angle, f_fv, 0.75, check_orientation=False)
    assert m1[3] == -1 and m1[5] == 2


def test_oracle_descriptor_distance_quirk():
    lib = oracle_lib.load()
    a = np.zeros(32, np.uint8)
    b = np.full(32, 0xFF, np.uint8)
    assert lib.oracle_descriptor_distance(oracle_lib._p(a), oracle_lib._p(b)) == 256
    assert lib.oracle_line_descriptor_distance(oracle_lib._p(a), oracle_lib._p(b)) == 128
    b[:4] = [1, 0, 0, 0]
    b[4:] = 0
    assert lib.oracle_descriptor_distance(oracle_lib._p(a), oracle_lib._p(b)) == 1
    assert lib.oracle_line_descriptor_distance(oracle_lib._p(a), oracle_lib._p(b)) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("nnratio,ori", [(0.7, True), (0.75, True), (0.6, False)])
def test_search_by_bow_matches_oracle(seed, nnratio, ori):
    import plvi
    case = util.bow_case(seed, n_kf=700 + 37 * seed, n_f=900 + 11 * seed)
    n_ref, m_ref = oracle_lib.search_by_bow(*case, nnratio, ori)
    n, m = plvi.ORBmatcher(nnratio, ori).SearchByBoW(*case)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)
    assert n_ref > 50  # the synthetic case does exercise matching


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("nleft_frac,ori", [(0.5, True), (0.3, False), (1.0, True), (0.0, True)])
def test_search_by_bow_two_cameras_matches_oracle(seed, nleft_frac, ori):
    import plvi
    case = util.bow_case(40 + seed, n_kf=600 + 29 * seed, n_f=900 + 17 * seed, dup=0.8)
    nleft = int(nleft_frac * len(case[4]))
    n_ref, m_ref = oracle_lib.search_by_bow(*case, 0.75, ori, f_nleft=nleft)
    n, m = plvi.ORBmatcher(0.75, ori).SearchByBoW(*case, f_nleft=nleft)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)
    # nLeft == 0: every feature is a right-camera one, the left best never passes TH_LOW -> no match at all
    assert n_ref == 0 if nleft == 0 else n_ref > 30


@pytest.mark.gpu
def test_search_by_bow_edge_cases():
    import plvi
    rng = np.random.default_rng(1)
    kf = _desc(rng, 5)
    f = np.concatenate([kf[:3], kf[:3]])  # exact duplicates: ties -> ratio test fails
    ang = np.zeros(5, np.float32)
    fang = np.zeros(6, np.float32)
    live = np.ones(5, np.uint8)
    for kf_fv, f_fv in [({1: [0, 1, 2, 3, 4]}, {1: [0, 1, 2, 3, 4, 5]}), ({1: [0, 1]}, {2: [0, 1, 2, 3, 4, 5]}),
                        ({}, {2: [0, 1, 2, 3, 4, 5]}), ({3: [4], 5: [0, 1, 2, 3]}, {5: [0, 3], 6: [1, 2, 4, 5]})]:
        ref = oracle_lib.search_by_bow(kf, ang, live, kf_fv, f, fang, f_fv, 0.7, True)
        got = plvi.ORBmatcher(0.7, True).SearchByBoW(kf, ang, live, kf_fv, f, fang, f_fv)
        assert got[0] == ref[0]
        np.testing.assert_array_equal(got[1], ref[1])


@pytest.mark.gpu
def test_descriptor_distance_batch_both_quirks():
    import plvi
    rng = np.random.default_rng(3)
    a, b = _desc(rng, 1000), _desc(rng, 1000)
    lib = oracle_lib.load()
    ref24 = [lib.oracle_descriptor_distance(oracle_lib._p(a[i]), oracle_lib._p(b[i])) for i in range(1000)]
    ref25 = [lib.oracle_line_descriptor_distance(oracle_lib._p(a[i]), oracle_lib._p(b[i])) for i in range(1000)]
    np.testing.assert_array_equal(plvi.ORBmatcher.DescriptorDistance(a, b), ref24)
    np.testing.assert_array_equal(plvi.ORBmatcher.DescriptorDistance(a, b, True), ref25)


@pytest.mark.gpu
def test_search_by_bow_batch_device():
    """plvi_search_by_bow_batch: several (KF, F) pairs in one launch, fixed capacities."""
    import ctypes
    import plvi
    lib = plvi.load()
    cases = [util.bow_case(40 + i, n_kf=300 + 50 * i, n_f=400 + 30 * i, n_nodes=60) for i in range(3)]
    P, kcap, fcap, ncap = len(cases), 500, 500, 64
    kd = np.zeros((P, kcap, 32), np.uint8); ka = np.zeros((P, kcap), np.float32); kl = np.zeros((P, kcap), np.uint8)
    fd = np.zeros((P, fcap, 32), np.uint8); fa = np.zeros((P, fcap), np.float32); fnk = np.zeros(P, np.int32)
    kn = np.zeros((P, ncap), np.int32); ko = np.zeros((P, ncap + 1), np.int32); kc = np.zeros(P, np.int32)
    ki = np.zeros((P, kcap), np.int32)
    fn = np.zeros((P, ncap), np.int32); fo = np.zeros((P, ncap + 1), np.int32); fc = np.zeros(P, np.int32)
    fi = np.zeros((P, fcap), np.int32)
    refs = []
    for p, c in enumerate(cases):
        kdesc, kang, klive, kfv, fdesc, fang, ffv = c
        kd[p, :len(kdesc)] = kdesc; ka[p, :len(kang)] = kang; kl[p, :len(klive)] = klive
        fd[p, :len(fdesc)] = fdesc; fa[p, :len(fang)] = fang; fnk[p] = len(fdesc)
        a, b, cidx = plvi.feature_vector_csr(kfv)
        kn[p, :len(a)] = a; ko[p, :len(b)] = b; kc[p] = len(a); ki[p, :len(cidx)] = cidx
        a, b, cidx = plvi.feature_vector_csr(ffv)
        fn[p, :len(a)] = a; fo[p, :len(b)] = b; fc[p] = len(a); fi[p, :len(cidx)] = cidx
        refs.append(oracle_lib.search_by_bow(*c, 0.75, True))
    bufs = []
    def dev(a):
        b = plvi.DeviceBuffer(max(a.nbytes, 4)); b.upload(np.ascontiguousarray(a)); bufs.append(b)
        return ctypes.c_void_p(b.ptr)
    out = plvi.DeviceBuffer(P * fcap * 4); cnt = plvi.DeviceBuffer(P * 4)
    rc = lib.plvi_search_by_bow_batch(P, 0.75, 1, kcap, fcap, ncap, dev(kd), dev(ka), dev(kl), dev(kn), dev(ko),
                                      dev(kc), dev(ki), dev(fd), dev(fa), dev(fnk), dev(fn), dev(fo), dev(fc),
                                      dev(fi), ctypes.c_void_p(out.ptr), ctypes.c_void_p(cnt.ptr), None)
    assert rc == 0
    lib.plvi_device_synchronize()
    m = out.download(np.zeros((P, fcap), np.int32))
    n = cnt.download(np.zeros(P, np.int32))
    for p, (n_ref, m_ref) in enumerate(refs):
        assert n[p] == n_ref
        np.testing.assert_array_equal(m[p, :len(m_ref)], m_ref)
