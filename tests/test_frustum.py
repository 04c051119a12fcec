"""The local-map visibility test: Frame::isInFrustum / isInFrustumChecks /
isInFrustum_l and MapPoint::PredictScale (src/Frame.cc:758-933, :1751-1824;
src/MapPoint.cc:502-546; src/MapLine.cc:384-394) as Tracking::SearchLocalPoints
and SearchLocalPointsAndLines call them (src/Tracking.cc:5074-5092,
:5166-5184, :5214-5292), and the line filter after LineMatcher::match.

The reference has no tests for these.  What is pinned: the fused sites and
instruction sequences of Frame.cc.o / MapPoint.cc.o (tests/test_ref_objects.py:
mTrackProjXR = fma(-mbf, invz, u), the four isInFrustum_l endpoint
coordinates, logf -> vdivss -> vroundss -> vcvttss2si in PredictScale, the
double division of viewCos).  Parity unpinned: OpenCV's own gemm / norm / dot
arithmetic (oracle/frustum_oracle.cpp header; PLVI_COMPAT_GEMM_FMA switches
the gemm contraction).  CPU: the C oracle against a numpy restatement, the
PredictScale table against logf over every float ratio of the level range.
GPU: the HIP kernels through the C-ABI bit-exactly against the oracle, and
chained on the device into the local searches (flags / proj / level in the
layout search_local_kernel reads; compacted descriptors into
plvi_line_match_batch, then the filter)."""
import ctypes

import numpy as np
import pytest

import oracle_lib
import util

LEVEL_CONFIGS = [(8, 1.2), (12, 1.2), (2, 2.0), (16, 1.1), (4, 1.5), (1, 1.2)]


def _same(a, b):
    """Bit-equal, or both NaN (the NaN sign / payload of 0/0 is the producer's)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        u = a.view(np.uint32 if a.dtype == np.float32 else np.uint64)
        v = b.view(u.dtype)
        return bool(np.all((u == v) | (np.isnan(a) & np.isnan(b))))
    return np.array_equal(a, b)


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("nlevels,scale", LEVEL_CONFIGS)
def test_level_table_equals_predict_scale(nlevels, scale):
    """level = #{n : ratio >= level_ratio[n]} equals ceil(logf(ratio)/lsf) clamped, for every float ratio
    in [2^-3, 2^(log2(scale)*nlevels + 2)] (all thresholds and beyond)."""
    import plvi
    p = plvi.FrustumParams()
    p.nlevels = nlevels
    p.log_scale_factor = float(np.float32(np.log(np.float32(scale))))
    plvi.frustum_params_init(p)
    thr = np.array(p.level_ratio[:], np.float32)
    assert np.all(np.isinf(thr[nlevels:])) and np.all(np.diff(thr[1:nlevels]) > 0)
    hi = float(2.0 ** (np.log2(scale) * nlevels + 2))
    bad, first = oracle_lib.level_table_check(thr, p.log_scale_factor, nlevels, 0.125, hi)
    assert bad == 0, hex(first)
    for n in range(1, nlevels):  # the threshold is the first float with level n
        t = thr[n]
        assert oracle_lib.predict_scale(float(t), 1.0, p.log_scale_factor, nlevels) == n
        below = np.nextafter(t, np.float32(0))
        assert oracle_lib.predict_scale(float(below), 1.0, p.log_scale_factor, nlevels) == n - 1


def test_predict_scale_special_ratios():
    """max/0 = inf -> ceil(inf) -> cvttss2si INT_MIN -> 0; 0/0 = NaN -> 0; ratio < 1 -> 0; huge -> n-1."""
    lsf = float(np.float32(np.log(np.float32(1.2))))
    assert oracle_lib.predict_scale(5.0, 0.0, lsf, 8) == 0
    assert oracle_lib.predict_scale(0.0, 0.0, lsf, 8) == 0
    assert oracle_lib.predict_scale(1.0, 2.0, lsf, 8) == 0
    assert oracle_lib.predict_scale(1e30, 1e-6, lsf, 8) == 7
    assert oracle_lib.predict_scale(1.0, 1.0, lsf, 8) == 0  # logf(1) = 0 -> ceil 0


def test_frustum_params_init_arguments():
    import plvi
    p = plvi.FrustumParams()
    p.log_scale_factor = 0.18
    for nl in (0, 17, -1):
        p.nlevels = nl
        with pytest.raises(plvi.PlviError):
            plvi.frustum_params_init(p)
    p.nlevels = 8
    p.log_scale_factor = -0.1
    with pytest.raises(plvi.PlviError):
        plvi.frustum_params_init(p)
    p.log_scale_factor = 0.0  # scale factor 1: logf(r)/0 is +-inf / NaN -> INT_MIN -> level 0 always
    plvi.frustum_params_init(p)
    assert all(np.isinf(v) for v in p.level_ratio[1:])
    for r in (0.5, 1.0, 3.0, 1e30):
        assert oracle_lib.predict_scale(r, 1.0, 0.0, 8) == 0


def test_frustum_wrappers_refuse_short_arrays():
    """The C entry points copy n records from every host array: a shorter one raises ValueError in the
    wrapper before any copy (no GPU needed)."""
    import plvi
    p = plvi.FrustumParams()
    n = 5
    pos, nrm, dst, fl = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros((n, 2)), np.ones(n, np.uint8)
    for kw in (dict(normal=nrm[:4]), dict(dist=dst[:3]), dict(in_flags=fl[:1]), dict(level=np.zeros(4)),
               dict(depth=np.zeros(6)), dict(proj=np.zeros((2, 4)))):
        args = dict(normal=nrm, dist=dst, in_flags=fl)
        args.update(kw)
        with pytest.raises(ValueError):
            plvi.frustum_points(p, pos, args["normal"], args["dist"], args["in_flags"],
                                **{k: v for k, v in kw.items() if k not in ("normal", "dist", "in_flags")})
    sep = np.zeros((n, 6))
    for kw in (dict(normal=nrm[:4]), dict(desc=np.zeros((3, 32), np.uint8)), dict(angle=np.zeros(2))):
        args = dict(normal=nrm, dist=dst, in_flags=fl)
        args.update(kw)
        with pytest.raises(ValueError):
            plvi.frustum_lines(p, sep, args["normal"], args["dist"], args["in_flags"],
                               **{k: v for k, v in kw.items() if k not in ("normal", "dist", "in_flags")})


def _numpy_is_in_frustum(p, case):
    """Frame.cc:760-835 (Pinhole, compat 0) in numpy float32 / float64: one IEEE op per operator, the
    Frame.cc.o fused mTrackProjXR via util.fmaf, PredictScale via the oracle's logf."""
    f32, f64 = np.float32, np.float64
    c = p.cam[0]
    R = np.array(c.R[:], f32).reshape(3, 3)
    t = np.array(c.t[:], f32)
    O = np.array(c.O[:], f32)
    out = []
    for i in range(len(case["pos"])):
        if not case["in_flags"][i] & 1:
            out.append(None)
            continue
        P = case["pos"][i].astype(f32)
        pc = np.array([f32(f64(f32(f32(R[r, 0] * P[0]) + f32(R[r, 1] * P[1])) + f32(R[r, 2] * P[2])) + f64(t[r]))
                       for r in range(3)], f32)
        pc_dist = f32(np.sqrt(f64(pc[0]) ** 2 + f64(pc[1]) ** 2 + f64(pc[2]) ** 2))
        with np.errstate(all="ignore"):
            invz = f32(f32(1) / pc[2])
            if pc[2] < 0:
                out.append(("behind",))
                continue
            u = f32(f32(f32(c.fx) * pc[0]) / pc[2]) + f32(c.cx)
            v = f32(f32(f32(c.fy) * pc[1]) / pc[2]) + f32(c.cy)
        if u < f32(p.min_x) or u > f32(p.max_x) or v < f32(p.min_y) or v > f32(p.max_y):
            out.append(("bounds",))
            continue
        mn, mx = case["dist"][i]
        PO = (P - O).astype(f32)
        dist = f32(np.sqrt((f64(PO[0]) ** 2 + f64(PO[1]) ** 2) + f64(PO[2]) ** 2))
        if dist < f32(f32(0.8) * mn) or dist > f32(f32(1.2) * mx):
            out.append(("dist", u, v))
            continue
        n = case["normal"][i]
        with np.errstate(all="ignore"):
            vc = f32((f64(PO[0]) * f64(n[0]) + f64(PO[1]) * f64(n[1]) + f64(PO[2]) * f64(n[2])) / f64(dist))
        if vc < f32(p.view_cos_limit):
            out.append(("cos", u, v))
            continue
        lvl = oracle_lib.predict_scale(float(mx), float(dist), p.log_scale_factor, p.nlevels)
        out.append(("in", u, v, util.fmaf(-f32(p.mbf), invz, u), vc, lvl, pc_dist))
    return out


def test_oracle_points_match_numpy_restatement():
    p = util.frustum_params(3)
    case = util.frustum_case(3, p, n=1500)
    got = oracle_lib.frustum_points(p, case)
    exp = _numpy_is_in_frustum(p, case)
    kinds = {}
    for i, e in enumerate(exp):
        fl = got["flags"][i]
        if e is None:
            assert fl == case["in_flags"][i] & 2
            continue
        kinds[e[0]] = kinds.get(e[0], 0) + 1
        if e[0] == "in":
            assert fl & 8 and fl & 16 and fl & 1, i
            pr = got["proj"][i]
            assert _same(pr, np.array([e[1], e[2], e[3], e[4]], np.float32)), (i, pr, e)
            assert got["level"][i] == e[5] and _same(got["depth"][i], e[6])
        else:
            assert not fl & (1 | 8 | 16), i
            if e[0] in ("behind", "bounds"):
                assert got["proj"][i][0] == -1 and got["proj"][i][1] == -1
            else:
                assert _same(got["proj"][i][:2], np.array(e[1:3], np.float32))
            assert _same(got["proj"][i][2:], case["proj"][i][2:]) and got["level"][i] == case["level"][i]
    assert got["nvisible"] == kinds.get("in", 0)
    assert all(kinds.get(k, 0) > 20 for k in ("in", "behind", "bounds", "dist", "cos")), kinds
    assert len(set(got["level"][got["flags"] & 8 > 0])) == 8


def test_oracle_degenerate_points():
    """Camera-centre points: Pc = 0 -> u = 0/0 NaN passes the bounds tests (NaN compares false), dist 0
    passes with mfMinDistance 0, viewCos 0/0 NaN passes the limit, max/0 = inf -> level 0."""
    import plvi
    p = plvi.FrustumParams()
    c = p.cam[0]
    c.R[0] = c.R[4] = c.R[8] = 1.0
    c.fx, c.fy, c.cx, c.cy = 400.0, 400.0, 320.0, 240.0
    p.min_x, p.max_x, p.min_y, p.max_y = 0.0, 640.0, 0.0, 480.0
    p.view_cos_limit, p.nlevels, p.log_scale_factor = 0.5, 8, float(np.float32(np.log(np.float32(1.2))))
    plvi.frustum_params_init(p)
    case = {"pos": np.array([[0, 0, 0], [1, 0, 0], [0, 0, 2]], np.float32),
            "normal": np.array([[0, 0, 1]] * 3, np.float32), "dist": np.array([[0, 5], [0, 5], [0, 0]], np.float32),
            "in_flags": np.array([3, 1, 1], np.uint8), "proj": np.zeros((3, 4), np.float32),
            "level": np.full(3, 5, np.int32), "depth": np.zeros(3, np.float32),
            "proj_r": np.zeros((3, 4), np.float32), "level_r": np.zeros(3, np.int32)}
    got = oracle_lib.frustum_points(p, case)
    assert got["flags"][0] == 1 | 2 | 8 | 16 and np.isnan(got["proj"][0][0]) and got["level"][0] == 0
    assert got["flags"][1] == 0 and got["proj"][1][0] == -1  # z == 0: u = +inf fails the bounds
    assert got["flags"][2] == 0  # mfMaxDistance 0: dist 2 > 0


def test_oracle_lines_sanity():
    p = util.frustum_params(5)
    case = util.frustum_line_case(5, p)
    iv, pr, an, cp = oracle_lib.frustum_lines(p, case)
    assert 50 < len(cp) < len(iv) and np.array_equal(cp, np.nonzero(iv)[0])
    # in-view angles are atan2f of the stored projections
    for i in cp[:50]:
        assert an[i] == np.float64(np.float32(np.arctan2(np.float64(pr[i, 3] - pr[i, 1]),
                                                         np.float64(pr[i, 2] - pr[i, 0])))) or \
            abs(an[i] - np.arctan2(pr[i, 3] - pr[i, 1], pr[i, 2] - pr[i, 0])) < 1e-6


# ------------------------------------------------------------------ GPU
POINT_CASES = [(0, False, False, 0), (0, False, True, 0), (0, False, False, 8), (1, False, False, 0),
               (0, True, False, 0), (1, True, True, 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("model,two,far,compat", POINT_CASES)
def test_frustum_points_match_oracle(model, two, far, compat):
    import plvi
    for seed in (0, 1):
        p = util.frustum_params(10 + seed, model=model, two_camera=two, far_points=far, compat=compat)
        case = util.frustum_case(20 + seed, p)
        exp = oracle_lib.frustum_points(p, case)
        nv, fl, pr, lv, de, prr, lvr = plvi.frustum_points(p, case["pos"], case["normal"], case["dist"],
                                                           case["in_flags"], case["proj"], case["level"],
                                                           case["depth"], case["proj_r"], case["level_r"])
        assert nv == exp["nvisible"] > 100
        assert _same(fl, exp["flags"]) and _same(pr, exp["proj"]) and _same(lv, exp["level"])
        assert _same(de, exp["depth"])
        if two:
            assert _same(prr, exp["proj_r"]) and _same(lvr, exp["level_r"])


@pytest.mark.gpu
def test_frustum_points_degenerate():
    import plvi
    p = util.frustum_params(0)
    nv, fl, *_ = plvi.frustum_points(p, np.zeros((0, 3)), np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.uint8))
    assert nv == 0 and len(fl) == 0
    case = util.frustum_case(1, p, n=6)
    exp = oracle_lib.frustum_points(p, case)
    nv, fl, pr, lv, de, _, _ = plvi.frustum_points(p, case["pos"], case["normal"], case["dist"], case["in_flags"],
                                                   case["proj"], case["level"], case["depth"])
    assert nv == exp["nvisible"] and _same(fl, exp["flags"]) and _same(pr, exp["proj"])


def _dev(bufs, a):
    import plvi
    a = np.ascontiguousarray(a)
    b = plvi.DeviceBuffer(max(a.nbytes, 4))
    if a.nbytes:
        b.upload(a)
    bufs.append(b)
    return ctypes.c_void_p(b.ptr)


def _keypoints_near(rng, proj, level, n_extra, W, H):
    """Current-frame keypoints at the predicted projections (+ noise) with octave ~ level, plus clutter."""
    import plvi
    m = len(proj)
    k = np.zeros(m + n_extra, plvi.KEYPOINT_DTYPE)
    k["x"][:m] = proj[:, 0] + rng.normal(0, 1.2, m)
    k["y"][:m] = proj[:, 1] + rng.normal(0, 1.2, m)
    k["octave"][:m] = np.clip(level + rng.integers(-1, 1, m), 0, 7)
    k["x"][m:] = rng.uniform(0, W, n_extra)
    k["y"][m:] = rng.uniform(0, H, n_extra)
    k["octave"][m:] = np.minimum(rng.geometric(0.35, n_extra) - 1, 7)
    k["size"] = 31
    k["class_id"] = -1
    perm = rng.permutation(len(k))
    return k[perm], perm


@pytest.mark.gpu
@pytest.mark.parametrize("two", [False, True])
def test_frustum_feeds_local_search_on_device(two):
    """frustum_points_batch -> assign_grid_batch -> search_local(_stereo)_batch with no host step between, vs
    the oracle chain oracle_frustum_points -> oracle_search_local(2)."""
    import plvi
    lib = plvi.load()
    rng = np.random.default_rng(7)
    # LDS of the two-camera search: 16 B per MapPoint + ~17 B per keypoint per side <= 160 KB
    F, cap, kcap, nmp = 3, 2600, (2300 if two else 3200), (1700 if two else 2400)
    ps, cases, kps_l, descs = [], [], [], []
    for f in range(F):
        p = util.frustum_params(30 + f, two_camera=two, far_points=(f == 1))
        case = util.frustum_case(40 + f, p, n=nmp + 50 * f)
        e = oracle_lib.frustum_points(p, case)
        vis = np.nonzero(e["flags"] & 1)[0]
        k, perm = _keypoints_near(rng, e["proj"][vis], e["level"][vis], 300, 752, 480)
        mdesc = rng.integers(0, 256, (len(case["pos"]), 32), dtype=np.uint8)
        kd = np.zeros((len(k), 32), np.uint8)
        src = np.full(len(k), -1)
        src[:len(vis)] = vis
        src = src[perm]
        bits = np.unpackbits(mdesc[np.maximum(src, 0)], axis=1)
        bits ^= (rng.random(bits.shape) < 0.06).astype(np.uint8)
        kd[:] = np.where((src >= 0)[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (len(k), 32)))
        ps.append(p); cases.append((case, e, mdesc)); kps_l.append(k); descs.append(kd)
    prm = (plvi.FrustumParams * F)(*ps)
    bufs = []
    # MapPoint tables [F][cap]
    pos = np.zeros((F, cap, 3), np.float32); nrm = np.zeros((F, cap, 3), np.float32)
    dst = np.zeros((F, cap, 2), np.float32); fin = np.zeros((F, cap), np.uint8)
    pr = np.zeros((F, cap, 4), np.float32); lv = np.zeros((F, cap), np.int32); de = np.zeros((F, cap), np.float32)
    prr = np.zeros((F, cap, 4), np.float32); lvr = np.zeros((F, cap), np.int32)
    md = np.zeros((F, cap, 32), np.uint8); mn = np.zeros(F, np.int32)
    kk = np.zeros((F, kcap), plvi.KEYPOINT_DTYPE); kdd = np.zeros((F, kcap, 32), np.uint8)
    kn = np.zeros(F, np.int32); kb = np.zeros((F, kcap), np.uint8)
    for f, (case, _, mdesc) in enumerate(cases):
        n = len(case["pos"])
        pos[f, :n] = case["pos"]; nrm[f, :n] = case["normal"]; dst[f, :n] = case["dist"]
        fin[f, :n] = case["in_flags"]; pr[f, :n] = case["proj"]; lv[f, :n] = case["level"]
        de[f, :n] = case["depth"]; prr[f, :n] = case["proj_r"]; lvr[f, :n] = case["level_r"]
        md[f, :n] = mdesc; mn[f] = n
        kk[f, :len(kps_l[f])] = kps_l[f]; kdd[f, :len(kps_l[f])] = descs[f]; kn[f] = len(kps_l[f])
        kb[f, :len(kps_l[f])] = (rng.random(len(kps_l[f])) < 0.04)
    d_prm = _dev(bufs, np.frombuffer(bytes(prm), np.uint8))
    d_fl = _dev(bufs, np.zeros((F, cap), np.uint8))
    d_pr, d_lv, d_de = _dev(bufs, pr), _dev(bufs, lv), _dev(bufs, de)
    d_prr, d_lvr = _dev(bufs, prr), _dev(bufs, lvr)
    d_nv = _dev(bufs, np.zeros(F, np.int32))
    d_mn = _dev(bufs, mn)
    rc = lib.plvi_frustum_points_batch(F, d_prm, _dev(bufs, pos), _dev(bufs, nrm), _dev(bufs, dst), _dev(bufs, fin),
                                       d_mn, cap, d_fl, d_pr, d_lv, d_prr if two else None, d_lvr if two else None,
                                       d_de, d_nv, None)
    assert rc == 0
    d_k, d_kn = _dev(bufs, kk), _dev(bufs, kn)
    off = plvi.DeviceBuffer(F * 3073 * 4); idx = plvi.DeviceBuffer(F * kcap * 4)
    g = plvi.grid_geometry(752, 480)
    lp = plvi.LocalParams()
    lp.min_x, lp.min_y, lp.inv_w, lp.inv_h, lp.th, lp.nnratio, lp.nlevels = g[0], g[2], g[4], g[5], 3.0, 0.8, 8
    for i, s in enumerate(util.orb_scale_factors()):
        lp.scale_factors[i] = s
    d_match = _dev(bufs, np.zeros((F, kcap), np.int32)); d_nm = _dev(bufs, np.zeros(F, np.int32))
    if not two:
        plvi.assign_grid_batch(d_k.value, d_kn.value, kcap, F, plvi.GridParams(g[0], g[2], g[4], g[5]), off.ptr,
                               idx.ptr)
        rc = lib.plvi_search_local_batch(F, ctypes.byref(lp), d_k, _dev(bufs, kdd), d_kn, kcap, _dev(bufs, kb), None,
                                         ctypes.c_void_p(off.ptr), ctypes.c_void_p(idx.ptr), d_fl, d_pr, d_lv,
                                         _dev(bufs, md), d_mn, cap, d_match, d_nm, None)
        assert rc == 0
    else:
        # right camera = the same keypoints (a rig seeing the same pattern): grids of both sides
        off_r = plvi.DeviceBuffer(F * 3073 * 4); idx_r = plvi.DeviceBuffer(F * kcap * 4)
        for o, ix in ((off, idx), (off_r, idx_r)):
            plvi.assign_grid_batch(d_k.value, d_kn.value, kcap, F, plvi.GridParams(g[0], g[2], g[4], g[5]), o.ptr,
                                   ix.ptr)
        d_match_r = _dev(bufs, np.zeros((F, kcap), np.int32))
        rc = lib.plvi_search_local_stereo_batch(
            F, ctypes.byref(lp), d_k, _dev(bufs, kdd), d_kn, kcap, _dev(bufs, kb), None, ctypes.c_void_p(off.ptr),
            ctypes.c_void_p(idx.ptr), d_k, _dev(bufs, kdd), d_kn, kcap, _dev(bufs, kb), None,
            ctypes.c_void_p(off_r.ptr), ctypes.c_void_p(idx_r.ptr), d_fl, d_pr, d_lv, d_prr, d_lvr, _dev(bufs, md),
            d_mn, cap, d_match, d_match_r, d_nm, None)
        assert rc == 0
    lib.plvi_device_synchronize()
    nv = plvi.download(d_nv.value, np.zeros(F, np.int32))
    match = plvi.download(d_match.value, np.zeros((F, kcap), np.int32))
    nm = plvi.download(d_nm.value, np.zeros(F, np.int32))
    if two:
        match_r = plvi.download(d_match_r.value, np.zeros((F, kcap), np.int32))
    for f, (case, e, mdesc) in enumerate(cases):
        assert nv[f] == e["nvisible"]
        ocase = {"cur_kps": kps_l[f], "cur_desc": descs[f], "cur_blocked": kb[f, :kn[f]], "cur_uright": None,
                 "grid": g, "scale_factors": util.orb_scale_factors(), "mp_flags": e["flags"],
                 "mp_proj": e["proj"], "mp_level": e["level"], "mp_desc": mdesc}
        if not two:
            ne, me = oracle_lib.search_local(ocase, 3.0, 0.8)
            assert nm[f] == ne > 50
            np.testing.assert_array_equal(match[f, :kn[f]], me)
        else:
            sc = {"kps": kps_l[f], "desc": descs[f], "kps_r": kps_l[f], "desc_r": descs[f],
                  "blocked": kb[f, :kn[f]], "blocked_r": kb[f, :kn[f]], "l2r": np.full(kn[f], -1),
                  "r2l": np.full(kn[f], -1), "grid": g,
                  "scale_factors": util.orb_scale_factors(), "mp_flags": e["flags"], "mp_proj": e["proj"],
                  "mp_level": e["level"], "mp_proj_r": e["proj_r"], "mp_level_r": e["level_r"], "mp_desc": mdesc}
            ne, ml, mr = oracle_lib.search_local_stereo(sc, 3.0, 0.8)
            assert nm[f] == ne > 50
            np.testing.assert_array_equal(match[f, :kn[f]], ml)
            np.testing.assert_array_equal(match_r[f, :kn[f]], mr)


@pytest.mark.gpu
@pytest.mark.parametrize("compat", [0, 8])
def test_frustum_lines_match_oracle(compat):
    import plvi
    for seed in (0, 1, 2):
        p = util.frustum_params(50 + seed, compat=compat)
        case = util.frustum_line_case(60 + seed, p)
        iv, pr, an, cp = oracle_lib.frustum_lines(p, case)
        giv, gpr, gan, gcp, gcd = plvi.frustum_lines(p, case["sep"], case["normal"], case["dist"], case["in_flags"],
                                                     case["desc"], case["proj"], case["angle"])
        assert len(cp) > 50
        assert _same(giv, iv) and _same(gpr, pr) and _same(gan, an) and _same(gcp, cp)
        assert np.array_equal(gcd, case["desc"][cp])


@pytest.mark.gpu
def test_frustum_lines_feed_match_and_filter_on_device():
    """frustum_lines_batch -> line_match_batch (compacted descriptors vs the frame's) ->
    local_lines_filter_batch, vs oracle_frustum_lines -> LineMatcher::match -> the Tracking.cc filter."""
    import plvi
    lib = plvi.load()
    rng = np.random.default_rng(11)
    F, cap, kcap = 3, 900, 700
    ps, cases, kls, kds, blks = [], [], [], [], []
    for f in range(F):
        p = util.frustum_params(70 + f)
        case = util.frustum_line_case(80 + f, p, n=850)
        iv, pr, an, cp = oracle_lib.frustum_lines(p, case)
        # frame keylines: noisy copies of most in-view projections (some flipped / shifted), plus clutter
        m = len(cp)
        kl = np.zeros(m + 150, oracle_lib.KEYLINE_DTYPE)
        q = pr[cp] + rng.normal(0, 4, (m, 4)) * (rng.random((m, 1)) < 0.8) + \
            rng.normal(0, 80, (m, 4)) * (rng.random((m, 1)) < 0.1)
        flip = rng.random(m) < 0.1
        q[flip] = q[flip][:, [2, 3, 0, 1]]
        kl["startPointX"][:m], kl["startPointY"][:m], kl["endPointX"][:m], kl["endPointY"][:m] = q.T
        c = rng.uniform(0, 752, (150, 4))
        kl["startPointX"][m:], kl["startPointY"][m:], kl["endPointX"][m:], kl["endPointY"][m:] = c.T
        bits = np.unpackbits(case["desc"][cp], axis=1)
        bits ^= (rng.random(bits.shape) < 0.05).astype(np.uint8)
        kd = np.concatenate([np.packbits(bits, axis=1), rng.integers(0, 256, (150, 32), dtype=np.uint8)])
        perm = rng.permutation(len(kl))
        kl, kd = kl[perm], kd[perm]
        ps.append(p); cases.append((case, iv, pr, an, cp)); kls.append(kl); kds.append(kd)
        blks.append((rng.random(len(kl)) < 0.05).astype(np.uint8))
    prm = (plvi.FrustumParams * F)(*ps)
    bufs = []
    sep = np.zeros((F, cap, 6)); nrm = np.zeros((F, cap, 3), np.float32); dst = np.zeros((F, cap, 2), np.float32)
    fin = np.zeros((F, cap), np.uint8); des = np.zeros((F, cap, 32), np.uint8); n = np.zeros(F, np.int32)
    pr0 = np.zeros((F, cap, 4), np.float32); an0 = np.zeros((F, cap))
    K = np.zeros((F, kcap), oracle_lib.KEYLINE_DTYPE); KD = np.zeros((F, kcap, 32), np.uint8)
    KN = np.zeros(F, np.int32); BL = np.zeros((F, kcap), np.uint8)
    for f, (case, *_r) in enumerate(cases):
        m = len(case["sep"])
        sep[f, :m] = case["sep"]; nrm[f, :m] = case["normal"]; dst[f, :m] = case["dist"]
        fin[f, :m] = case["in_flags"]; des[f, :m] = case["desc"]; n[f] = m
        pr0[f, :m] = case["proj"]; an0[f, :m] = case["angle"]
        K[f, :len(kls[f])] = kls[f]; KD[f, :len(kls[f])] = kds[f]; KN[f] = len(kls[f]); BL[f, :len(kls[f])] = blks[f]
    d = lambda a: _dev(bufs, a)  # noqa: E731
    d_prm = d(np.frombuffer(bytes(prm), np.uint8))
    d_iv, d_pr, d_an = d(np.zeros((F, cap), np.uint8)), d(pr0), d(an0)
    d_cp, d_cd, d_nc = d(np.zeros((F, cap), np.int32)), d(np.zeros((F, cap, 32), np.uint8)), d(np.zeros(F, np.int32))
    rc = lib.plvi_frustum_lines_batch(F, d_prm, d(sep), d(nrm), d(dst), d(fin), d(des), d(n), cap, d_iv, d_pr, d_an,
                                      d_cp, d_cd, d_nc, None)
    assert rc == 0
    d_kn = d(KN)
    d_scr = d(np.zeros(4 * F * (cap + kcap), np.int32))
    d_m12, d_nmt = d(np.zeros((F, cap), np.int32)), d(np.zeros(F, np.int32))
    rc = lib.plvi_line_match_batch(d_cd, d_nc, cap, d(KD), d_kn, kcap, F, ctypes.c_float(0.9), d_scr, d_m12, d_nmt,
                                   None)
    assert rc == 0
    d_as, d_na = d(np.zeros((F, kcap), np.int32)), d(np.zeros(F, np.int32))
    rc = lib.plvi_local_lines_filter_batch(F, d_prm, d_m12, d_nc, d_cp, cap, d_pr, d_an, d(K), d_kn, kcap, d(BL),
                                           d_as, d_na, None)
    assert rc == 0
    lib.plvi_device_synchronize()
    get = lambda ptr, like: plvi.download(ptr.value, like)  # noqa: E731
    nc = get(d_nc, np.zeros(F, np.int32))
    m12 = get(d_m12, np.zeros((F, cap), np.int32))
    asg = get(d_as, np.zeros((F, kcap), np.int32))
    na = get(d_na, np.zeros(F, np.int32))
    for f, (case, iv, pr, an, cp) in enumerate(cases):
        assert nc[f] == len(cp)
        _, em = oracle_lib.match(case["desc"][cp], kds[f], 0.9)
        ena, easg, em_after = oracle_lib.local_lines_filter(ps[f], em, cp, pr, an, kls[f], blks[f])
        assert na[f] == ena > 20
        np.testing.assert_array_equal(asg[f, :len(kls[f])], easg)
        np.testing.assert_array_equal(m12[f, :len(cp)], em_after)
