"""ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
const set<MapPoint*>& sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:2180-2300)
-- the relocalization guided search Tracking::Relocalization runs for every
candidate KeyFrame while tracking is lost (src/Tracking.cc:5857 with th 10 /
ORBdist 100, :5871 with th 3 / ORBdist 64; ORBmatcher(0.9, true)).

Parity unpinned: the reference has no tests for it.  The C++ oracle
(oracle/proj_oracle.cpp: oracle_search_reloc) restates the cited lines and is
checked here against a pure-Python restatement; the HIP path
(search_reloc_kernel, csrc/proj.hip) is compared with the oracle exactly
(match table incl. the rotation filter's NULLs, nmatches)."""
import math

import numpy as np
import pytest

import oracle_lib
import util

f32 = np.float32


def _py_reloc(case, th, orb_dist, check_ori=True):
    """Pure-Python restatement of ORBmatcher.cc:2180-2300 (float32 arithmetic where the reference uses float)."""
    k = case["cur_kps"]
    n_cur = len(k)
    min_x, max_x, min_y, max_y, inv_w, inv_h = case["grid"]
    cells = [[[] for _ in range(48)] for _ in range(64)]
    for i in range(n_cur):  # AssignFeaturesToGrid / PosInGrid (std::round: half away from zero)
        gx, gy = f32(f32(k["x"][i] - min_x) * inv_w), f32(f32(k["y"][i] - min_y) * inv_h)
        px = int(math.floor(gx + 0.5)) if gx >= 0 else -int(math.floor(-gx + 0.5))
        py = int(math.floor(gy + 0.5)) if gy >= 0 else -int(math.floor(-gy + 0.5))
        if 0 <= px < 64 and 0 <= py < 48:
            cells[px][py].append(i)
    fx, fy, cx, cy, _ = case["camera"]
    sf = case["scale_factors"]
    nonnull = case["cur_blocked"].astype(bool).copy()
    mp = np.full(n_cur, -1, np.int32)
    hist = [[] for _ in range(30)]
    nm = 0
    for i in range(len(case["kf_flags"])):
        if not case["kf_flags"][i] & 1:
            continue
        xc, yc, zc = (f32(t) for t in case["x3dc"][i])
        u = f32(f32(f32(fx * xc) / zc) + cx)
        v = f32(f32(f32(fy * yc) / zc) + cy)
        if u < min_x or u > max_x or v < min_y or v > max_y:
            continue
        d3, dmin, dmax = (f32(t) for t in case["dist"][i])
        if d3 < dmin or d3 > dmax:
            continue
        L = int(case["level"][i])
        if L < 0 or L >= len(sf):
            continue
        r = f32(f32(th) * f32(sf[L]))
        x0 = max(0, math.floor(f32(f32(u - min_x) - r) * inv_w))
        x1 = min(63, math.ceil(f32(f32(u - min_x) + r) * inv_w))
        y0 = max(0, math.floor(f32(f32(v - min_y) - r) * inv_h))
        y1 = min(47, math.ceil(f32(f32(v - min_y) + r) * inv_h))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        cand = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for i2 in cells[ix][iy]:
                    o = k["octave"][i2]
                    if o < L - 1 or o > L + 1:
                        continue
                    if abs(f32(k["x"][i2] - u)) < r and abs(f32(k["y"][i2] - v)) < r:
                        cand.append(i2)
        best, bi = 256, -1
        for i2 in cand:
            if nonnull[i2]:
                continue
            d = int(np.unpackbits(case["mp_desc"][i] ^ case["cur_desc"][i2]).sum())
            if d < best:
                best, bi = d, i2
        if bi >= 0 and best <= orb_dist:
            mp[bi] = i
            nonnull[bi] = True
            nm += 1
            if check_ori:
                rot = f32(case["kf_angle"][i] - k["angle"][bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                q = f32(rot * f32(1.0 / 30))
                b = int(math.floor(q + 0.5))  # roundf, q >= 0
                hist[0 if b == 30 else b].append(bi)
    if check_ori:
        m1 = m2 = m3 = 0
        i1 = i2_ = i3 = -1
        for b in range(30):
            c = len(hist[b])
            if c > m1:
                m3, m2, m1, i3, i2_, i1 = m2, m1, c, i2_, i1, b
            elif c > m2:
                m3, m2, i3, i2_ = m2, c, i2_, b
            elif c > m3:
                m3, i3 = c, b
        if m2 < f32(0.1) * f32(m1):
            i2_ = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for b in range(30):
            if b not in (i1, i2_, i3):
                for idx in hist[b]:
                    mp[idx] = -2
                    nm -= 1
    return nm, mp


@pytest.mark.parametrize("seed,th,orb_dist,ori", [(0, 10.0, 100, True), (1, 3.0, 64, True), (2, 10.0, 100, False)])
def test_oracle_reloc_matches_python(seed, th, orb_dist, ori):
    case = util.reloc_case(seed, n_cur=300, n_kf=240)
    n, m = oracle_lib.search_reloc(case, th, orb_dist, int(ori))
    ne, me = _py_reloc(case, th, orb_dist, ori)
    assert n == ne
    np.testing.assert_array_equal(m, me)
    assert n > 20


def test_oracle_reloc_sanity():
    case = util.reloc_case(5)
    n, m = oracle_lib.search_reloc(case, 10.0, 100)
    assert n > 100 and (m == -2).sum() > 0
    assert (m[case["cur_blocked"] == 1] == -1).all()  # mvpMapPoints already set: never overwritten
    kept = np.nonzero(m >= 0)[0]
    assert len(set(m[kept])) == len(kept)  # one keypoint per MapPoint
    for i2 in kept:
        d = int(np.unpackbits(case["mp_desc"][m[i2]] ^ case["cur_desc"][i2]).sum())
        assert d <= 100
    n3, m3 = oracle_lib.search_reloc(case, 3.0, 64)
    assert 0 < n3 < n


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("th,orb_dist,ori", [(10.0, 100, True), (3.0, 64, True), (10.0, 100, False),
                                             (25.0, 255, True), (1.0, 0, True)])
def test_search_reloc_matches_oracle(seed, th, orb_dist, ori):
    import plvi
    case = util.reloc_case(20 + seed, n_cur=1000 + 41 * seed, n_kf=800 + 13 * seed)
    n_ref, m_ref = oracle_lib.search_reloc(case, th, orb_dist, int(ori))
    p = util.reloc_params(case, th, orb_dist)
    n, m = plvi.ORBmatcher(0.9, ori).SearchByProjectionKF(
        p, case["cur_kps"], case["cur_desc"], case["kf_flags"], case["x3dc"], case["dist"], case["level"],
        case["kf_angle"], case["mp_desc"], case["cur_blocked"])
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


@pytest.mark.gpu
def test_search_reloc_degenerate():
    import plvi
    case = util.reloc_case(9, n_cur=60, n_kf=5)
    mt = plvi.ORBmatcher(0.9, True)
    for nkf in (0, 1, 5):
        c = dict(case)
        for key in ("kf_flags", "x3dc", "dist", "level", "kf_angle", "mp_desc"):
            c[key] = case[key][:nkf]
        for blk in (case["cur_blocked"], np.ones(60, np.uint8)):
            c["cur_blocked"] = blk
            ne, me = oracle_lib.search_reloc(c, 10.0, 100)
            ng, mg = mt.SearchByProjectionKF(util.reloc_params(c, 10.0, 100), c["cur_kps"], c["cur_desc"],
                                             c["kf_flags"], c["x3dc"], c["dist"], c["level"], c["kf_angle"],
                                             c["mp_desc"], c["cur_blocked"])
            assert ng == ne and np.array_equal(mg, me)
    bad = util.reloc_params(case, 10.0, 256)  # ORBdist 256 would index mvpMapPoints[-1] in the reference
    with pytest.raises(RuntimeError):
        mt.SearchByProjectionKF(bad, case["cur_kps"], case["cur_desc"], case["kf_flags"], case["x3dc"],
                                case["dist"], case["level"], case["kf_angle"], case["mp_desc"])


@pytest.mark.gpu
def test_search_reloc_batch_device():
    """Several candidate KeyFrames against one current frame in one launch (the relocalization loop's
    candidates), grid built on the device."""
    import ctypes
    import plvi
    lib = plvi.load()
    cases = [util.reloc_case(60 + i, n_cur=700 + 90 * i, n_kf=500 + 70 * i) for i in range(4)]
    P, cc, kc = len(cases), 1000, 800
    kp = np.zeros((P, cc), plvi.KEYPOINT_DTYPE); cd = np.zeros((P, cc, 32), np.uint8)
    cb = np.zeros((P, cc), np.uint8); cn = np.zeros(P, np.int32)
    fl = np.zeros((P, kc), np.uint8); x3 = np.zeros((P, kc, 3), np.float32); ds = np.zeros((P, kc, 3), np.float32)
    lv = np.zeros((P, kc), np.int32); an = np.zeros((P, kc), np.float32); md = np.zeros((P, kc, 32), np.uint8)
    kn = np.zeros(P, np.int32)
    for p, c in enumerate(cases):
        n, m = len(c["cur_kps"]), len(c["kf_flags"])
        kp[p, :n] = c["cur_kps"]; cd[p, :n] = c["cur_desc"]; cb[p, :n] = c["cur_blocked"]; cn[p] = n
        fl[p, :m] = c["kf_flags"]; x3[p, :m] = c["x3dc"]; ds[p, :m] = c["dist"]; lv[p, :m] = c["level"]
        an[p, :m] = c["kf_angle"]; md[p, :m] = c["mp_desc"]; kn[p] = m
    bufs = []

    def dev(a):
        b = plvi.DeviceBuffer(max(a.nbytes, 4)); b.upload(np.ascontiguousarray(a)); bufs.append(b)
        return b.ptr
    off = plvi.DeviceBuffer(P * 3073 * 4); idx = plvi.DeviceBuffer(P * cc * 4)
    g = cases[0]["grid"]
    dk, dn = dev(kp), dev(cn)
    plvi.assign_grid_batch(dk, dn, cc, P, plvi.GridParams(g[0], g[2], g[4], g[5]), off.ptr, idx.ptr)
    prm = util.reloc_params(cases[0], 10.0, 100)
    prm.check_orientation = 1
    out = plvi.DeviceBuffer(P * cc * 4); nm = plvi.DeviceBuffer(P * 4)
    V = ctypes.c_void_p
    rc = lib.plvi_search_reloc_batch(P, ctypes.byref(prm), V(dk), V(dev(cd)), V(dn), cc, V(dev(cb)), V(off.ptr),
                                     V(idx.ptr), V(dev(fl)), V(dev(x3)), V(dev(ds)), V(dev(lv)), V(dev(an)),
                                     V(dev(md)), V(dev(kn)), kc, V(out.ptr), V(nm.ptr), None)
    assert rc == 0
    lib.plvi_device_synchronize()
    M = out.download(np.zeros((P, cc), np.int32)); N = nm.download(np.zeros(P, np.int32))
    for p, c in enumerate(cases):
        n_ref, m_ref = oracle_lib.search_reloc(c, 10.0, 100)
        assert N[p] == n_ref
        np.testing.assert_array_equal(M[p, :len(m_ref)], m_ref)
