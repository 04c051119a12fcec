"""ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th, bFarPoints, thFarPoints) on a
two-camera Frame (F.Nleft != -1, src/ORBmatcher.cc:44-214): the local-map search of stereo KannalaBrandt8
rigs.  Left keypoints (mvKeys) in mGrid, right keypoints (mvKeysRight) in mGridRight with right-relative
indices (src/Frame.cc:644-675, GetFeaturesInArea(..., bRight) :1006-1075); a MapPoint is searched in each
image it is predicted in, assignments are mirrored into the stereo partner (mvLeftToRightMatch /
mvRightToLeftMatch), and a left ratio-test failure skips the MapPoint's right search (the `continue` at :127).

Parity unpinned: the reference has no tests for it.  The C++ oracle (oracle/proj_oracle.cpp:
oracle_search_local2) restates the cited lines and is checked here against a pure-Python restatement; the
HIP path (search_local2_kernel, csrc/proj.hip) is compared with the oracle exactly (both match tables incl.
overwrites, nmatches).

Reference quirks encoded by both: a left ratio-test failure `continue`s past the right search
(ORBmatcher.cc:126-127); the far-point test reads the left mTrackDepth for both images (:56; stale when only
the right camera sees the point -- plvi_frustum_points_batch keeps that value, tests/test_frustum.py)."""
import math

import numpy as np
import pytest

import oracle_lib
import util
from test_projection import _py_grid

f32 = np.float32


def _py_in_area(cells, k, grid, x, y, r, lo, hi):
    min_x, _, min_y, _, inv_w, inv_h = grid
    x0 = max(0, math.floor(f32(f32(x - min_x) - r) * inv_w))
    if x0 >= 64:
        return []
    x1 = min(63, math.ceil(f32(f32(x - min_x) + r) * inv_w))
    if x1 < 0:
        return []
    y0 = max(0, math.floor(f32(f32(y - min_y) - r) * inv_h))
    if y0 >= 48:
        return []
    y1 = min(47, math.ceil(f32(f32(y - min_y) + r) * inv_h))
    if y1 < 0:
        return []
    check = lo > 0 or hi >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in cells[ix][iy]:
                o = k["octave"][i]
                if check and (o < lo or (hi >= 0 and o > hi)):
                    continue
                if abs(f32(k["x"][i] - x)) < r and abs(f32(k["y"][i] - y)) < r:
                    out.append(i)
    return out


def _py_local_stereo(c, th, nnratio=0.8):
    """Pure-Python restatement of ORBmatcher.cc:44-214 with F.Nleft != -1."""
    kl, kr = c["kps"], c["kps_r"]
    nl, nr = len(kl), len(kr)
    cl = _py_grid(kl["x"], kl["y"], c["grid"])
    cr = _py_grid(kr["x"], kr["y"], c["grid"])
    desc = np.concatenate([c["desc"], c["desc_r"]])
    blocked = np.concatenate([c["blocked"], c["blocked_r"]]).astype(bool)
    match = np.full(nl + nr, -1, np.int32)
    sf = c["scale_factors"]
    nm = 0

    def dist(m, i):
        return int(np.unpackbits(c["mp_desc"][m] ^ desc[i]).sum())

    def store(i, m):
        match[i] = m
        blocked[i] = bool(c["mp_flags"][m] & 2)

    def best_of(idxs, m, off, oct_):
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for idx in idxs:
            if blocked[idx + off]:
                continue
            d = dist(m, idx + off)
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(oct_[idx]), idx
            elif d < bd2:
                bl2, bd2 = int(oct_[idx]), d
        return bd, bl, bd2, bl2, bi

    for m in range(len(c["mp_flags"])):
        fl = int(c["mp_flags"][m])
        if not fl & 5:
            continue
        if fl & 1:
            L = int(c["mp_level"][m])
            r = f32(2.5) if c["mp_proj"][m, 3] > 0.998 else f32(4.0)
            if th != 1.0:
                r = f32(r * f32(th))
            rad = f32(r * f32(sf[L]))
            idxs = _py_in_area(cl, kl, c["grid"], c["mp_proj"][m, 0], c["mp_proj"][m, 1], rad, L - 1, L)
            if idxs:
                bd, bl, bd2, bl2, bi = best_of(idxs, m, 0, kl["octave"])
                if bd <= 100:
                    if bl == bl2 and bd > f32(nnratio) * bd2:
                        continue
                    store(bi, m)
                    if c["l2r"][bi] != -1:
                        store(int(c["l2r"][bi]) + nl, m)
                        nm += 1
                    nm += 1
        if fl & 4:
            L = int(c["mp_level_r"][m])
            if L != -1:
                r = f32(2.5) if c["mp_proj_r"][m, 3] > 0.998 else f32(4.0)
                rad = f32(r * f32(sf[L]))
                idxs = _py_in_area(cr, kr, c["grid"], c["mp_proj_r"][m, 0], c["mp_proj_r"][m, 1], rad, L - 1, L)
                if not idxs:
                    continue
                bd, bl, bd2, bl2, bi = best_of(idxs, m, nl, kr["octave"])
                if bd <= 100:
                    if bl == bl2 and bd > f32(nnratio) * bd2:
                        continue
                    if c["r2l"][bi] != -1:
                        store(int(c["r2l"][bi]), m)
                        nm += 1
                    store(bi + nl, m)
                    nm += 1
    return nm, match[:nl], match[nl:]


@pytest.mark.parametrize("seed,th", [(0, 1.0), (1, 3.0)])
def test_oracle_local_stereo_matches_python(seed, th):
    case = util.local_stereo_case(seed, n_left=300, n_right=280, n_mp=450)
    n, ml, mr = oracle_lib.search_local_stereo(case, th)
    ne, mle, mre = _py_local_stereo(case, th)
    assert n == ne
    np.testing.assert_array_equal(ml, mle)
    np.testing.assert_array_equal(mr, mre)
    assert n > 100


def test_oracle_local_stereo_sanity():
    case = util.local_stereo_case(4)
    n, ml, mr = oracle_lib.search_local_stereo(case, 1.0)
    assert (ml >= 0).sum() > 200 and (mr >= 0).sum() > 150
    # a blocked keypoint is never a candidate; it only receives a MapPoint as the stereo partner of a match
    # (the reference overwrites mvpMapPoints[mvLeftToRightMatch[idx] + Nleft] unchecked, :133 / :200)
    bl = (case["blocked"] == 1) & (ml >= 0)
    br = (case["blocked_r"] == 1) & (mr >= 0)
    assert (case["l2r"][bl] >= 0).all() and (case["r2l"][br] >= 0).all()
    # stereo mirroring: some MapPoints land on both keypoints of a pair
    pairs = np.nonzero(case["l2r"] >= 0)[0]
    assert (ml[pairs] >= 0).any() and ((ml[pairs] == mr[case["l2r"][pairs]]) & (ml[pairs] >= 0)).sum() > 20
    # right search off: only the left image (and mirrored right partners) receive MapPoints
    c = dict(case)
    c["mp_flags"] = case["mp_flags"] & 3
    n1, ml1, mr1 = oracle_lib.search_local_stereo(c, 1.0)
    assert set(np.nonzero(mr1 >= 0)[0]) <= set(case["l2r"][case["l2r"] >= 0])


def _gpu(case, th):
    import plvi
    mt = plvi.ORBmatcher(0.8, True)
    return mt.SearchByProjectionLocalStereo(util.local_params(case, th), case["kps"], case["desc"], case["kps_r"],
                                            case["desc_r"], case["mp_flags"], case["mp_proj"], case["mp_level"],
                                            case["mp_proj_r"], case["mp_level_r"], case["mp_desc"], case["blocked"],
                                            case["blocked_r"], case["l2r"], case["r2l"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,pair_frac", [(0, 1.0, 0.6), (1, 3.0, 0.6), (2, 1.0, 0.0), (3, 10.0, 0.9),
                                               (5, 5.0, 0.6)])
def test_local_stereo_matches_oracle(seed, th, pair_frac):
    case = util.local_stereo_case(20 + seed, pair_frac=pair_frac)
    ne, mle, mre = oracle_lib.search_local_stereo(case, th)
    ng, mlg, mrg = _gpu(case, th)
    assert ng == ne
    np.testing.assert_array_equal(mlg, mle)
    np.testing.assert_array_equal(mrg, mre)


@pytest.mark.gpu
def test_local_stereo_degenerate():
    """No MapPoints, one side empty, no stereo pairs (NULL tables), every keypoint blocked."""
    import plvi
    case = util.local_stereo_case(9, n_left=60, n_right=50, n_mp=40)
    mt = plvi.ORBmatcher(0.8, True)
    variants = []
    c = dict(case)
    for k in ("mp_flags", "mp_proj", "mp_level", "mp_proj_r", "mp_level_r", "mp_desc"):
        c[k] = case[k][:0]
    variants.append(c)
    c = dict(case)
    c["kps_r"], c["desc_r"], c["blocked_r"], c["r2l"] = case["kps_r"][:0], case["desc_r"][:0], case["blocked_r"][:0], \
        case["r2l"][:0]
    c["l2r"] = np.full(len(case["kps"]), -1, np.int32)
    variants.append(c)
    c = dict(case)
    c["blocked"], c["blocked_r"] = np.ones(60, np.uint8), np.ones(50, np.uint8)
    variants.append(c)
    for c in variants:
        ne, mle, mre = oracle_lib.search_local_stereo(c, 1.0)
        ng, mlg, mrg = mt.SearchByProjectionLocalStereo(util.local_params(c, 1.0), c["kps"], c["desc"], c["kps_r"],
                                                        c["desc_r"], c["mp_flags"], c["mp_proj"], c["mp_level"],
                                                        c["mp_proj_r"], c["mp_level_r"], c["mp_desc"], c["blocked"],
                                                        c["blocked_r"], c["l2r"], c["r2l"])
        assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre)
    # NULL pair tables = no stereo partner anywhere
    c = dict(case)
    c["l2r"] = np.full(60, -1, np.int32)
    c["r2l"] = np.full(50, -1, np.int32)
    ne, mle, mre = oracle_lib.search_local_stereo(c, 1.0)
    ng, mlg, mrg = mt.SearchByProjectionLocalStereo(util.local_params(c, 1.0), c["kps"], c["desc"], c["kps_r"],
                                                    c["desc_r"], c["mp_flags"], c["mp_proj"], c["mp_level"],
                                                    c["mp_proj_r"], c["mp_level_r"], c["mp_desc"], c["blocked"],
                                                    c["blocked_r"])
    assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre)


@pytest.mark.gpu
def test_local_stereo_batch_device():
    """Several two-camera frames in one launch through plvi_search_local_stereo_batch (device tables, both
    grids built on the device), each compared with the oracle."""
    import ctypes
    import plvi
    lib = plvi.load()
    cases = [util.local_stereo_case(70 + i, n_left=500 + 60 * i, n_right=450 + 50 * i, n_mp=700 + 80 * i)
             for i in range(3)]
    P, cl, cr, mc = len(cases), 700, 600, 900
    kl = np.zeros((P, cl), plvi.KEYPOINT_DTYPE); kr = np.zeros((P, cr), plvi.KEYPOINT_DTYPE)
    dl = np.zeros((P, cl, 32), np.uint8); dr = np.zeros((P, cr, 32), np.uint8)
    bl = np.zeros((P, cl), np.uint8); br = np.zeros((P, cr), np.uint8)
    l2r = np.full((P, cl), -1, np.int32); r2l = np.full((P, cr), -1, np.int32)
    nl = np.zeros(P, np.int32); nr = np.zeros(P, np.int32); nm = np.zeros(P, np.int32)
    fl = np.zeros((P, mc), np.uint8); pr = np.zeros((P, mc, 4), np.float32); lv = np.zeros((P, mc), np.int32)
    prr = np.zeros((P, mc, 4), np.float32); lvr = np.zeros((P, mc), np.int32); md = np.zeros((P, mc, 32), np.uint8)
    for p, c in enumerate(cases):
        a, b, m = len(c["kps"]), len(c["kps_r"]), len(c["mp_flags"])
        kl[p, :a] = c["kps"]; dl[p, :a] = c["desc"]; bl[p, :a] = c["blocked"]; l2r[p, :a] = c["l2r"]; nl[p] = a
        kr[p, :b] = c["kps_r"]; dr[p, :b] = c["desc_r"]; br[p, :b] = c["blocked_r"]; r2l[p, :b] = c["r2l"]
        nr[p] = b
        fl[p, :m] = c["mp_flags"]; pr[p, :m] = c["mp_proj"]; lv[p, :m] = c["mp_level"]
        prr[p, :m] = c["mp_proj_r"]; lvr[p, :m] = c["mp_level_r"]; md[p, :m] = c["mp_desc"]; nm[p] = m
    bufs = []

    def dev(x):
        b = plvi.DeviceBuffer(max(x.nbytes, 4)); b.upload(np.ascontiguousarray(x)); bufs.append(b)
        return b.ptr
    g = cases[0]["grid"]
    gp = plvi.GridParams(g[0], g[2], g[4], g[5])
    dkl, dnl, dkr, dnr = dev(kl), dev(nl), dev(kr), dev(nr)
    col = plvi.DeviceBuffer(P * 3073 * 4); cil = plvi.DeviceBuffer(P * cl * 4)
    cor = plvi.DeviceBuffer(P * 3073 * 4); cir = plvi.DeviceBuffer(P * cr * 4)
    plvi.assign_grid_batch(dkl, dnl, cl, P, gp, col.ptr, cil.ptr)
    plvi.assign_grid_batch(dkr, dnr, cr, P, gp, cor.ptr, cir.ptr)
    prm = util.local_params(cases[0], 1.0)
    prm.nnratio = 0.8
    ml = plvi.DeviceBuffer(P * cl * 4); mr = plvi.DeviceBuffer(P * cr * 4); nmt = plvi.DeviceBuffer(P * 4)
    V = ctypes.c_void_p
    rc = lib.plvi_search_local_stereo_batch(P, ctypes.byref(prm), V(dkl), V(dev(dl)), V(dnl), cl, V(dev(bl)),
                                            V(dev(l2r)), V(col.ptr), V(cil.ptr), V(dkr), V(dev(dr)), V(dnr), cr,
                                            V(dev(br)), V(dev(r2l)), V(cor.ptr), V(cir.ptr), V(dev(fl)), V(dev(pr)),
                                            V(dev(lv)), V(dev(prr)), V(dev(lvr)), V(dev(md)), V(dev(nm)), mc,
                                            V(ml.ptr), V(mr.ptr), V(nmt.ptr), None)
    assert rc == 0
    lib.plvi_device_synchronize()
    ML = ml.download(np.zeros((P, cl), np.int32)); MR = mr.download(np.zeros((P, cr), np.int32))
    N = nmt.download(np.zeros(P, np.int32))
    for p, c in enumerate(cases):
        ne, mle, mre = oracle_lib.search_local_stereo(c, 1.0)
        assert N[p] == ne
        np.testing.assert_array_equal(ML[p, :len(mle)], mle)
        np.testing.assert_array_equal(MR[p, :len(mre)], mre)
