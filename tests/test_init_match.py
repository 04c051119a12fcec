"""The monocular initializer's matchers (Tracking::MonocularInitialization,
src/Tracking.cc:3111-3113): ORBmatcher::SearchForInitialization
(src/ORBmatcher.cc:705-814) and LineMatcher::SerachForInitialize
(src/LineMatcher.cpp:113-139) with Frame::lineDescriptorMAD
(src/Frame.cc:1089-1112).

Parity unpinned: the reference ships no tests for them.  The C++ oracle is
checked against pure-Python restatements here (the window in the
reference's cell order, the sequential vMatchedDistance / steal logic, the
rotation filter; the MAD medians by sorting the match lists with the
reference's comparators), and the HIP path is compared with the oracle
exactly (vnMatches12, nmatches, the updated vbPrevMatched; LineMatches
pairs and the MAD values) on frames extracted by the oracle itself."""
import math

import numpy as np
import pytest

import oracle_lib as ol
from plvi import synth

F32 = np.float32
W, H = 640, 480
GRID = (F32(0), F32(0), F32(64) / F32(W), F32(48) / F32(H))


def _seq(n, seed):
    return synth.device_sequence(n, W, H, seed=seed).numpy()


_cache = {}


def _orb(img_key, img):
    if img_key not in _cache:
        _, k, d = ol.orb_extract(img)
        _cache[img_key] = (k, d)
    return _cache[img_key]


def _lines(img_key, img):
    if ("l",) + img_key not in _cache:
        kl, d, _ = ol.line_extract(img)
        _cache[("l",) + img_key] = d
    return _cache[("l",) + img_key]


def _pos_in_grid(x, y):
    fx = F32(F32(x - GRID[0]) * GRID[2])
    fy = F32(F32(y - GRID[1]) * GRID[3])
    rnd = lambda v: int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))  # noqa: E731
    return rnd(float(fx)), rnd(float(fy))


def _py_search_init(k1, d1, prev, k2, d2, window=100, nnratio=F32(0.9), check=True):
    """Pure-Python SearchForInitialization (ORBmatcher.cc:705-814)."""
    cells = [[[] for _ in range(48)] for _ in range(64)]
    for i in range(len(k2)):
        px, py = _pos_in_grid(k2["x"][i], k2["y"][i])
        if 0 <= px < 64 and 0 <= py < 48:
            cells[px][py].append(i)
    n1, n2 = len(k1), len(k2)
    m12 = [-1] * n1
    m21 = [-1] * n2
    md = [2 ** 31 - 1] * n2
    hist = [[] for _ in range(30)]
    nm = 0
    pop = lambda a, b: int(np.unpackbits(np.bitwise_xor(a, b)).sum())  # noqa: E731
    r = F32(window)
    for i1 in range(n1):
        if k1["octave"][i1] > 0:
            continue
        x, y = F32(prev[i1][0]), F32(prev[i1][1])
        x0 = max(0, math.floor(F32(F32(x - GRID[0]) - r) * GRID[2]))
        x1 = min(63, math.ceil(F32(F32(x - GRID[0]) + r) * GRID[2]))
        y0 = max(0, math.floor(F32(F32(y - GRID[1]) - r) * GRID[3]))
        y1 = min(47, math.ceil(F32(F32(y - GRID[1]) + r) * GRID[3]))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        idx = [i for ix in range(x0, x1 + 1) for iy in range(y0, y1 + 1) for i in cells[ix][iy]
               if k2["octave"][i] == 0 and abs(F32(k2["x"][i] - x)) < r and abs(F32(k2["y"][i] - y)) < r]
        if not idx:
            continue
        b, b2, bi = 2 ** 31 - 1, 2 ** 31 - 1, -1
        for i2 in idx:
            dd = pop(d1[i1], d2[i2])
            if md[i2] <= dd:
                continue
            if dd < b:
                b2, b, bi = b, dd, i2
            elif dd < b2:
                b2 = dd
        if b <= 50 and F32(b) < F32(F32(b2) * nnratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1], m21[bi], md[bi] = bi, i1, b
            nm += 1
            if check:
                rot = F32(k1["angle"][i1] - k2["angle"][bi])
                if rot < 0:
                    rot = F32(rot + F32(360))
                v = float(F32(rot * F32(F32(1) / F32(30))))
                binv = int(math.floor(v + 0.5))
                hist[0 if binv == 30 else binv].append(i1)
    if check:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i_1 = i_2 = i_3 = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i_3, i_2, i_1 = m2, m1, s, i_2, i_1, i
            elif s > m2:
                m3, m2, i_3, i_2 = m2, s, i_2, i
            elif s > m3:
                m3, i_3 = s, i
        if m2 < F32(0.1) * F32(m1):
            i_2 = i_3 = -1
        elif m3 < F32(0.1) * F32(m1):
            i_3 = -1
        for i in range(30):
            if i in (i_1, i_2, i_3):
                continue
            for j in hist[i]:
                if m12[j] >= 0:
                    m12[j] = -1
                    nm -= 1
    pv = np.array(prev, np.float32).copy()
    for i1 in range(n1):
        if m12[i1] >= 0:
            pv[i1] = (k2["x"][m12[i1]], k2["y"][m12[i1]])
    return nm, np.array(m12, np.int32), pv


def _py_line_init(d1, d2):
    """Pure-Python SerachForInitialize + lineDescriptorMAD."""
    i0, a, _, b = ol.knn2(d1, d2)
    lm = [[i, int(i0[i]), F32(a[i]), F32(b[i])] for i in range(len(d1))]
    n = len(lm)
    nn = sorted(lm, key=lambda m: m[2])
    med = float(nn[n // 2][2])
    nn_mad = 1.4826 * float(sorted(F32(abs(float(m[2]) - med)) for m in nn)[n // 2])
    m12 = sorted(lm, key=lambda m: -(m[3] - m[2]))
    med12 = float(F32(m12[n // 2][3] - m12[n // 2][2]))
    nn12_mad = 1.4826 * float(sorted(F32(abs(float(F32(m[3] - m[2])) - med12)) for m in m12)[n // 2])
    th = nn12_mad * 0.5
    pairs = [(m[0], m[1]) for m in lm if float(F32(m[3] - m[2])) > th]
    return np.array(pairs, np.int32).reshape(-1, 2), (nn_mad, nn12_mad)


def _orb_pair(seed, gap):
    seq = _seq(gap + 1, seed)
    k1, d1 = _orb((seed, 0), seq[0])
    k2, d2 = _orb((seed, gap), seq[gap])
    return k1, d1, k2, d2


@pytest.mark.parametrize("seed,gap", [(3, 2), (11, 6)])
def test_oracle_search_for_initialization_matches_python(seed, gap):
    k1, d1, k2, d2 = _orb_pair(seed, gap)
    prev = np.stack([k1["x"], k1["y"]], 1)
    n, m, pv = ol.search_for_initialization(k1, d1, prev, k2, d2, GRID)
    pn, pm, ppv = _py_search_init(k1, d1, prev, k2, d2)
    assert n == pn and n > 20
    np.testing.assert_array_equal(m, pm)
    np.testing.assert_array_equal(pv, ppv)
    # second call with the updated vbPrevMatched (Tracking keeps it between frames)
    n2, m2, pv2 = ol.search_for_initialization(k1, d1, pv, k2, d2, GRID, window=30)
    pn2, pm2, ppv2 = _py_search_init(k1, d1, ppv, k2, d2, window=30)
    assert n2 == pn2
    np.testing.assert_array_equal(m2, pm2)
    np.testing.assert_array_equal(pv2, ppv2)


def test_oracle_search_for_initialization_steals_and_filters():
    """Known answers on a hand-built case: a later F1 keypoint with a smaller
    distance steals F2 keypoint 0 (vnMatches12 of the earlier one reset,
    nmatches unchanged); an equal distance does not (vMatchedDistance <=
    dist skips it); updated vbPrevMatched entries only for matches."""
    kp = np.dtype([("x", "<f4"), ("y", "<f4"), ("octave", "<i4"), ("angle", "<f4")])
    base = np.zeros(32, np.uint8)
    far = np.full(32, 0xFF, np.uint8)
    d2 = np.stack([base, far])
    k2 = np.array([(100, 100, 0, 10.0), (300, 300, 0, 10.0)], kp)
    one = base.copy()
    one[0] = 1
    two = base.copy()
    two[0] = 3
    d1 = np.stack([two, one, one, far])  # distances to F2[0]: 2, 1, 1; F2[1] far
    k1 = np.array([(100, 100, 0, 10.0), (101, 100, 0, 10.0), (102, 100, 0, 10.0), (300, 300, 1, 10.0)], kp)
    prev = np.stack([k1["x"], k1["y"]], 1)
    n, m, pv = ol.search_for_initialization(k1, d1, prev, k2, d2, GRID, check_ori=False)
    assert n == 1 and list(m) == [-1, 0, -1, -1]
    assert tuple(pv[1]) == (100.0, 100.0) and tuple(pv[2]) == (102.0, 100.0)
    pn, pm, _ = _py_search_init(k1, d1, prev, k2, d2, check=False)
    assert pn == n and list(pm) == list(m)


@pytest.mark.parametrize("seed,gap", [(5, 1), (9, 4)])
def test_oracle_line_search_init_matches_python(seed, gap):
    seq = _seq(gap + 1, seed)
    d1, d2 = _lines((seed, 0), seq[0]), _lines((seed, gap), seq[gap])
    pairs, mad = ol.line_search_init(d1, d2)
    pp, pmad = _py_line_init(d1, d2)
    assert len(pairs) > 5
    np.testing.assert_array_equal(pairs, pp)
    assert mad == pmad


def test_oracle_line_search_init_degenerate():
    d = np.zeros((1, 32), np.uint8)
    assert len(ol.line_search_init(np.zeros((0, 32), np.uint8), d)[0]) == 0
    assert len(ol.line_search_init(d, d)[0]) == 0  # one train line: undefined in the reference, no pairs
    # all queries equal: d1 - d0 == 32 everywhere -> median 32, nn12_mad 0,
    # every pair passes 32 > 0
    t = np.stack([np.zeros(32, np.uint8), np.full(32, 1, np.uint8)])
    pairs, mad = ol.line_search_init(np.zeros((5, 32), np.uint8), t)
    assert pairs.tolist() == [[i, 0] for i in range(5)] and mad == (0.0, 0.0)
    assert pairs.tolist() == _py_line_init(np.zeros((5, 32), np.uint8), t)[0].tolist()


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_search_for_initialization_batch_vs_oracle():
    """Several (F1, F2) pairs in one launch through the C-ABI batch entry
    point (device tables, grid by plvi_assign_grid_batch), two iterations of
    vbPrevMatched as Tracking carries it; each pair equals the oracle."""
    import plvi
    cases = [(3, 2), (11, 6), (21, 1), (30, 12)]
    pairs = [_orb_pair(s, g) for s, g in cases]
    P = len(pairs)
    cap1 = max(len(p[0]) for p in pairs)
    cap2 = max(len(p[2]) for p in pairs)
    K1 = np.zeros((P, cap1), plvi.KEYPOINT_DTYPE)
    K2 = np.zeros((P, cap2), plvi.KEYPOINT_DTYPE)
    D1 = np.zeros((P, cap1, 32), np.uint8)
    D2 = np.zeros((P, cap2, 32), np.uint8)
    PV = np.zeros((P, cap1, 2), np.float32)
    N = np.zeros(2 * P, np.int32)
    for i, (k1, d1, k2, d2) in enumerate(pairs):
        for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
            K1[i, :len(k1)][f] = k1[f]
            K2[i, :len(k2)][f] = k2[f]
        D1[i, :len(k1)] = d1
        D2[i, :len(k2)] = d2
        PV[i, :len(k1), 0], PV[i, :len(k1), 1] = k1["x"], k1["y"]
        N[i], N[P + i] = len(k1), len(k2)
    bufs = {k: plvi.DeviceBuffer(a.nbytes) for k, a in (("k1", K1), ("k2", K2), ("d1", D1), ("d2", D2), ("pv", PV),
                                                         ("n", N))}
    for k, a in (("k1", K1), ("k2", K2), ("d1", D1), ("d2", D2), ("pv", PV), ("n", N)):
        bufs[k].upload(a)
    co = plvi.DeviceBuffer(4 * 3073 * P)
    ci = plvi.DeviceBuffer(4 * cap2 * P)
    m = plvi.DeviceBuffer(4 * cap1 * P)
    nm = plvi.DeviceBuffer(4 * P)
    plvi.assign_grid_batch(bufs["k2"].ptr, bufs["n"].ptr + 4 * P, cap2, P, plvi.GridParams(*[float(g) for g in GRID]),
                           co.ptr, ci.ptr)
    prm = plvi.InitParams(*[float(g) for g in GRID], 100, 0.9, 1)
    ref_prev = [np.stack([p[0]["x"], p[0]["y"]], 1) for p in pairs]
    for it, win in enumerate((100, 40)):
        prm.window = win
        plvi.search_for_initialization_batch(P, prm, bufs["k1"].ptr, bufs["d1"].ptr, bufs["n"].ptr, cap1,
                                             bufs["pv"].ptr, bufs["k2"].ptr, bufs["d2"].ptr, bufs["n"].ptr + 4 * P,
                                             cap2, co.ptr, ci.ptr, m.ptr, nm.ptr)
        plvi.load().plvi_device_synchronize()
        gm = m.download(np.zeros((P, cap1), np.int32))
        gn = nm.download(np.zeros(P, np.int32))
        gpv = bufs["pv"].download(np.zeros((P, cap1, 2), np.float32))
        for i, (k1, d1, k2, d2) in enumerate(pairs):
            en, em, epv = ol.search_for_initialization(k1, d1, ref_prev[i], k2, d2, GRID, window=win)
            assert gn[i] == en and (it > 0 or en > 20), f"pair {i} iter {it}: {gn[i]} vs {en}"
            np.testing.assert_array_equal(gm[i, :len(k1)], em)
            np.testing.assert_array_equal(gpv[i, :len(k1)], epv)
            ref_prev[i] = epv


@pytest.mark.gpu
def test_search_for_initialization_host_edge_cases():
    """The host convenience path: no F2 keypoints, no level-0 F1 keypoints,
    the hand-built steal case, and far-away vbPrevMatched (empty windows)."""
    import plvi
    k1, d1, k2, d2 = _orb_pair(3, 2)
    prev = np.stack([k1["x"], k1["y"]], 1)
    n, m, pv = plvi.search_for_initialization(k1, d1, prev, k2[:0], d2[:0])
    assert n == 0 and (m == -1).all() and np.array_equal(pv, prev)
    hi = k1.copy()
    hi["octave"] = 1
    n, m, _ = plvi.search_for_initialization(hi, d1, prev, k2, d2)
    assert n == 0 and (m == -1).all()
    far = prev + np.float32(5000)
    n, m, _ = plvi.search_for_initialization(k1, d1, far, k2, d2)
    assert n == 0
    for check in (False, True):
        en, em, epv = ol.search_for_initialization(k1, d1, prev, k2, d2, GRID, check_ori=check)
        gn, gm, gpv = plvi.search_for_initialization(k1, d1, prev, k2, d2, check_orientation=check)
        assert gn == en
        np.testing.assert_array_equal(gm, em)
        np.testing.assert_array_equal(gpv, epv)


@pytest.mark.gpu
def test_line_search_init_batch_vs_oracle():
    """LineMatches and the MAD values of several pairs in one launch, plus
    the degenerate pairs (no query lines, one train line, all-equal rows)."""
    import plvi
    descs = []
    for seed, gap in ((5, 1), (9, 4), (14, 10)):
        seq = _seq(gap + 1, seed)
        descs.append((_lines((seed, 0), seq[0]), _lines((seed, gap), seq[gap])))
    z = np.zeros((5, 32), np.uint8)
    t2 = np.stack([np.zeros(32, np.uint8), np.full(32, 1, np.uint8)])
    descs += [(z[:0], t2), (z, t2[:1]), (z, t2)]
    P = len(descs)
    cap1 = max(max(len(a) for a, _ in descs), 1)
    cap2 = max(len(b) for _, b in descs)
    D1 = np.zeros((P, cap1, 32), np.uint8)
    D2 = np.zeros((P, cap2, 32), np.uint8)
    N = np.zeros(2 * P, np.int32)
    for i, (a, b) in enumerate(descs):
        D1[i, :len(a)] = a
        D2[i, :len(b)] = b
        N[i], N[P + i] = len(a), len(b)
    b1, b2, bn = plvi.DeviceBuffer(D1.nbytes), plvi.DeviceBuffer(D2.nbytes), plvi.DeviceBuffer(N.nbytes)
    b1.upload(D1)
    b2.upload(D2)
    bn.upload(N)
    scr = plvi.DeviceBuffer(16 * P * cap1)
    pr = plvi.DeviceBuffer(8 * P * cap1)
    cnt = plvi.DeviceBuffer(4 * P)
    mad = plvi.DeviceBuffer(16 * P)
    plvi.line_search_init_batch(b1.ptr, bn.ptr, cap1, b2.ptr, bn.ptr + 4 * P, cap2, P, scr.ptr, pr.ptr, cnt.ptr,
                                mad.ptr)
    plvi.load().plvi_device_synchronize()
    gp = pr.download(np.zeros((P, cap1, 2), np.int32))
    gc = cnt.download(np.zeros(P, np.int32))
    gm = mad.download(np.zeros((P, 2), np.float64))
    for i, (a, b) in enumerate(descs):
        ep, emad = ol.line_search_init(a, b)
        assert gc[i] == len(ep), f"pair {i}"
        np.testing.assert_array_equal(gp[i, :gc[i]], ep)
        if len(a) and len(b) >= 2:
            assert tuple(gm[i]) == emad
    assert gc[0] > 5
