"""Frame::AssignFeaturesToGrid / GetFeaturesInArea and
ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
(src/Frame.cc:644-675, 1006-1087; src/ORBmatcher.cc:1962-2178), SURVEY §8f
rank 2.

Parity unpinned: the reference has no tests for these; the C++ oracle
(oracle/proj_oracle.cpp) restates the cited lines, is checked here against
pure-Python restatements of the grid and the window query, and the HIP path
is compared with the oracle exactly (match table incl. overwrites and the
rotation filter's NULLs, nmatches)."""
import math

import numpy as np
import pytest

import oracle_lib
import util


def _py_grid(kx, ky, grid):
    min_x, max_x, min_y, max_y, inv_w, inv_h = grid
    cells = [[[] for _ in range(48)] for _ in range(64)]
    for i, (x, y) in enumerate(zip(kx, ky)):
        px = int(np.round(np.float32(np.float32(x - min_x) * inv_w)))
        py = int(np.round(np.float32(np.float32(y - min_y) * inv_h)))
        fx_ = np.float32(np.float32(x - min_x) * inv_w)
        fy_ = np.float32(np.float32(y - min_y) * inv_h)
        px = int(math.floor(fx_ + 0.5)) if fx_ >= 0 else -int(math.floor(-fx_ + 0.5))  # std::round: half away
        py = int(math.floor(fy_ + 0.5)) if fy_ >= 0 else -int(math.floor(-fy_ + 0.5))
        if 0 <= px < 64 and 0 <= py < 48:
            cells[px][py].append(i)
    return cells


def test_oracle_grid_matches_python():
    case = util.projection_case(1, n_cur=1500, n_last=10)
    k = case["cur_kps"]
    off, idx = oracle_lib.assign_grid(k["x"], k["y"], case["grid"])
    cells = _py_grid(k["x"], k["y"], case["grid"])
    flat = [i for ix in range(64) for iy in range(48) for i in cells[ix][iy]]
    assert list(idx) == flat
    counts = [len(cells[ix][iy]) for ix in range(64) for iy in range(48)]
    assert list(np.diff(off)) == counts


def test_oracle_features_in_area_matches_brute_force():
    case = util.projection_case(2, n_cur=1200, n_last=10)
    k = case["cur_kps"]
    rng = np.random.default_rng(0)
    f32 = np.float32
    for t in range(300):
        x, y = f32(rng.uniform(-30, 780)), f32(rng.uniform(-30, 510))
        r = f32(rng.choice([15, 30, 45, 100]) * rng.uniform(0.5, 3.6))
        lo, hi = [(int(rng.integers(-1, 8)), int(rng.integers(-1, 9))), (0, -1), (3, -1)][t % 3]
        got = oracle_lib.features_in_area(k["x"], k["y"], k["octave"], case["grid"], x, y, r, lo, hi)
        # brute force in the reference's cell order
        cells = _py_grid(k["x"], k["y"], case["grid"])
        min_x, max_x, min_y, max_y, inv_w, inv_h = case["grid"]
        x0 = max(0, math.floor(f32((x - min_x) - r) * inv_w))
        x1 = min(63, math.ceil(f32((x - min_x) + r) * inv_w))
        y0 = max(0, math.floor(f32((y - min_y) - r) * inv_h))
        y1 = min(47, math.ceil(f32((y - min_y) + r) * inv_h))
        exp = []
        if x0 < 64 and x1 >= 0 and y0 < 48 and y1 >= 0:
            check = lo > 0 or hi >= 0
            for ix in range(x0, x1 + 1):
                for iy in range(y0, y1 + 1):
                    for i in cells[ix][iy]:
                        o = k["octave"][i]
                        if check and (o < lo or (hi >= 0 and o > hi)):
                            continue
                        if abs(f32(k["x"][i] - x)) < r and abs(f32(k["y"][i] - y)) < r:
                            exp.append(i)
        assert list(got) == exp


def test_oracle_search_by_projection_known_answers():
    case = util.projection_case(3, n_cur=400, n_last=300)
    n, m = oracle_lib.search_by_projection(case, 15.0)
    assert n > 50 and (m >= 0).sum() > 50 and (m == -2).sum() > 0  # matches, and the 10-degree rotation filter bites
    # every kept match is within TH_HIGH and maps back to a valid point
    for i2 in np.nonzero(m >= 0)[0]:
        i = m[i2]
        assert case["flags"][i] & 1
        d = int(np.unpackbits(case["mp_desc"][i] ^ case["cur_desc"][i2]).sum())
        assert d <= 100
    n0, m0 = oracle_lib.search_by_projection(case, 15.0, check_ori=0)
    assert n0 >= n and (m0 == -2).sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("th,fwd,bwd,ori,ur", [(15.0, 0, 0, 1, False), (30.0, 0, 0, 1, False), (15.0, 1, 0, 1, True),
                                              (7.0, 0, 1, 0, True), (100.0, 0, 0, 1, False)])
def test_search_by_projection_matches_oracle(seed, th, fwd, bwd, ori, ur):
    import plvi
    case = util.projection_case(10 + seed, n_cur=1000 + 37 * seed, n_last=900 + 11 * seed, uright=ur)
    n_ref, m_ref = oracle_lib.search_by_projection(case, th, fwd, bwd, ori)
    p = util.proj_params(case, th, fwd, bwd)
    n, m = plvi.ORBmatcher(0.9, bool(ori)).SearchByProjection(
        p, case["cur_kps"], case["cur_desc"], case["x3dc"], case["last_octave"], case["last_angle"],
        case["mp_desc"], case["flags"], case["cur_blocked"], case["cur_uright"])
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)
    assert n_ref > 50


@pytest.mark.gpu
def test_assign_grid_and_projection_batch_device():
    import ctypes
    import plvi
    lib = plvi.load()
    cases = [util.projection_case(40 + i, n_cur=700 + 90 * i, n_last=600 + 50 * i) for i in range(3)]
    P, cc, lc = len(cases), 1000, 800
    kp = np.zeros((P, cc), plvi.KEYPOINT_DTYPE); cd = np.zeros((P, cc, 32), np.uint8)
    cb = np.zeros((P, cc), np.uint8); cn = np.zeros(P, np.int32)
    x3 = np.zeros((P, lc, 3), np.float32); lo = np.zeros((P, lc), np.int32); la = np.zeros((P, lc), np.float32)
    md = np.zeros((P, lc, 32), np.uint8); lf = np.zeros((P, lc), np.uint8); ln = np.zeros(P, np.int32)
    for p, c in enumerate(cases):
        n, m = len(c["cur_kps"]), len(c["flags"])
        kp[p, :n] = c["cur_kps"]; cd[p, :n] = c["cur_desc"]; cb[p, :n] = c["cur_blocked"]; cn[p] = n
        x3[p, :m] = c["x3dc"]; lo[p, :m] = c["last_octave"]; la[p, :m] = c["last_angle"]
        md[p, :m] = c["mp_desc"]; lf[p, :m] = c["flags"]; ln[p] = m
    bufs = []

    def dev(a):
        b = plvi.DeviceBuffer(max(a.nbytes, 4)); b.upload(np.ascontiguousarray(a)); bufs.append(b)
        return b.ptr
    off = plvi.DeviceBuffer(P * 3073 * 4); idx = plvi.DeviceBuffer(P * cc * 4)
    g = cases[0]["grid"]
    gp = plvi.GridParams(g[0], g[2], g[4], g[5])
    dk, dn = dev(kp), dev(cn)
    plvi.assign_grid_batch(dk, dn, cc, P, gp, off.ptr, idx.ptr)
    lib.plvi_device_synchronize()
    offs = off.download(np.zeros((P, 3073), np.int32)); idxs = idx.download(np.zeros((P, cc), np.int32))
    for p, c in enumerate(cases):
        eo, ei = oracle_lib.assign_grid(c["cur_kps"]["x"], c["cur_kps"]["y"], c["grid"])
        np.testing.assert_array_equal(offs[p], eo)
        np.testing.assert_array_equal(idxs[p, :len(ei)], ei)
    prm = util.proj_params(cases[0], 15.0)
    prm.check_orientation = 1
    out = plvi.DeviceBuffer(P * cc * 4); nm = plvi.DeviceBuffer(P * 4)
    V = ctypes.c_void_p
    rc = lib.plvi_search_by_projection_batch(P, ctypes.byref(prm), V(dk), V(dev(cd)), V(dn), cc, V(dev(cb)), None,
                                             V(off.ptr), V(idx.ptr), V(dev(x3)), V(dev(lo)), V(dev(la)), V(dev(md)),
                                             V(dev(lf)), V(dev(ln)), lc, V(out.ptr), V(nm.ptr), None)
    assert rc == 0
    lib.plvi_device_synchronize()
    M = out.download(np.zeros((P, cc), np.int32)); N = nm.download(np.zeros(P, np.int32))
    for p, c in enumerate(cases):
        n_ref, m_ref = oracle_lib.search_by_projection(c, 15.0)
        assert N[p] == n_ref
        np.testing.assert_array_equal(M[p, :len(m_ref)], m_ref)


# ------------------------------------------------- local-map search (ORBmatcher.cc:44-145)
def test_oracle_local_search_sanity():
    case = util.local_case(0)
    n, m = oracle_lib.search_local(case, 1.0)
    assert n > 200 and (m >= 0).sum() <= n
    # blocked keypoints never receive a MapPoint
    assert (m[case["cur_blocked"] == 1] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,uright", [(0, 1.0, False), (1, 3.0, False), (2, 1.0, True), (3, 10.0, False),
                                            (4, 1.0, False), (5, 5.0, True)])
def test_local_search_matches_oracle(seed, th, uright):
    import plvi
    case = util.local_case(seed, uright=uright)
    ne, me = oracle_lib.search_local(case, th, 0.8)
    mt = plvi.ORBmatcher(0.8, True)
    ng, mg = mt.SearchByProjectionLocal(util.local_params(case, th), case["cur_kps"], case["cur_desc"],
                                        case["mp_flags"], case["mp_proj"], case["mp_level"], case["mp_desc"],
                                        case["cur_blocked"], case["cur_uright"])
    assert ng == ne
    np.testing.assert_array_equal(mg, me)


@pytest.mark.gpu
def test_local_search_degenerate():
    import plvi
    case = util.local_case(9, n_cur=50, n_mp=1)
    mt = plvi.ORBmatcher(0.8, True)
    for nmp in (0, 1):
        c = dict(case)
        for k in ("mp_flags", "mp_proj", "mp_level", "mp_desc"):
            c[k] = case[k][:nmp]
        ne, me = oracle_lib.search_local(c, 1.0)
        ng, mg = mt.SearchByProjectionLocal(util.local_params(c, 1.0), c["cur_kps"], c["cur_desc"], c["mp_flags"],
                                            c["mp_proj"], c["mp_level"], c["mp_desc"], c["cur_blocked"])
        assert ng == ne and np.array_equal(mg, me)
