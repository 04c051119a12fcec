"""ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) with a two-camera
CurrentFrame (CurrentFrame.Nleft != -1, src/ORBmatcher.cc:1985-2175): every LastFrame point is projected by
CurrentFrame.mpCamera (KannalaBrandt8::project, CameraModels/KannalaBrandt8.cpp:33-48, or Pinhole) into the
left image and -- unless the left pass ended early -- into the right image (x3Dr = mTrl x3Dc, mGridRight);
both images' matches share one rotation histogram.

Parity unpinned: the reference has no tests for it.  The C++ oracle (oracle/proj_oracle.cpp:
oracle_search_by_projection2, host libm for atan2f / cosf / sinf as the reference calls them) restates the
cited lines; with a Pinhole rig it is checked here against the one-camera oracle on a frame whose right image
is empty, and its KannalaBrandt8 projection against a float64 model; the HIP path (search_by_projection2_kernel,
csrc/proj.hip, glibc atan2f / cosf / sinf restated in csrc/plvi_math.h) is compared with the oracle exactly
(both match tables incl. overwrites and the rotation filter's NULLs, nmatches).

Reference quirks the oracle and the kernel both encode (a change to either
must keep them): the right pass projects x3Dr with CurrentFrame.mpCamera, not
mpCamera2 (ORBmatcher.cc:2087); the right projection has no mnMin/MaxX/Y
bounds test (:2085-2093, unlike the left one at :2005-2008); the right window
uses the LastFrame point's own octave (:2089-2090)."""
import numpy as np
import pytest

import oracle_lib
import util


def test_oracle_stereo_projection_reduces_to_one_camera():
    """Pinhole rig, empty right image: the two-camera restatement equals the one-camera oracle."""
    c = util.projection_stereo_case(1, kb8=False)
    c["kps_r"], c["desc_r"], c["blocked_r"] = c["kps_r"][:0], c["desc_r"][:0], c["blocked_r"][:0]
    n2, ml, mr = oracle_lib.search_by_projection_stereo(c, 7.0)
    mono = {"cur_kps": c["kps"], "cur_desc": c["desc"], "cur_blocked": c["blocked"], "cur_uright": None,
            "grid": c["grid"], "scale_factors": c["scale_factors"], "x3dc": c["x3dc"], "flags": c["flags"],
            "last_octave": c["last_octave"], "last_angle": c["last_angle"], "mp_desc": c["mp_desc"],
            "camera": c["camera"]}
    n1, m1 = oracle_lib.search_by_projection(mono, 7.0)
    assert n2 == n1 and len(mr) == 0
    np.testing.assert_array_equal(ml, m1)
    assert n1 > 100


def test_oracle_stereo_projection_sanity():
    c = util.projection_stereo_case(2)
    n, ml, mr = oracle_lib.search_by_projection_stereo(c, 7.0)
    assert (ml >= 0).sum() > 150 and (mr >= 0).sum() > 80  # both images match
    assert (ml == -2).sum() + (mr == -2).sum() > 0          # the shared rotation filter bites
    assert n > 0 and n <= (ml != -1).sum() + (mr != -1).sum() + 200  # overwrites count in nmatches
    # Pinhole instead of KannalaBrandt8 on the same points: a different (fewer-match) answer, so the
    # fisheye projection is really used
    d = dict(c)
    d["kb8"] = None
    n0, ml0, _ = oracle_lib.search_by_projection_stereo(d, 7.0)
    assert not np.array_equal(ml0, ml)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,kb8,fb", [(0, 7.0, True, (0, 0)), (1, 15.0, True, (0, 0)), (2, 7.0, False, (0, 0)),
                                            (3, 7.0, True, (1, 0)), (4, 7.0, True, (0, 1)), (5, 3.0, True, (0, 0))])
def test_stereo_projection_matches_oracle(seed, th, kb8, fb):
    import plvi
    c = util.projection_stereo_case(30 + seed, kb8=kb8)
    ne, mle, mre = oracle_lib.search_by_projection_stereo(c, th, forward=fb[0], backward=fb[1])
    ng, mlg, mrg = plvi.ORBmatcher(0.9, True).SearchByProjectionStereo(
        util.proj_params(c, th, *fb), c["kps"], c["desc"], c["kps_r"], c["desc_r"], c["x3dc"], c["x3dr"],
        c["last_octave"], c["last_angle"], c["mp_desc"], c["flags"], c["kb8"], c["blocked"], c["blocked_r"])
    assert ng == ne
    np.testing.assert_array_equal(mlg, mle)
    np.testing.assert_array_equal(mrg, mre)


@pytest.mark.gpu
def test_stereo_projection_no_rotation_check_and_degenerate():
    import plvi
    c = util.projection_stereo_case(40)
    ne, mle, mre = oracle_lib.search_by_projection_stereo(c, 7.0, check_ori=0)
    ng, mlg, mrg = plvi.ORBmatcher(0.9, False).SearchByProjectionStereo(
        util.proj_params(c, 7.0), c["kps"], c["desc"], c["kps_r"], c["desc_r"], c["x3dc"], c["x3dr"],
        c["last_octave"], c["last_angle"], c["mp_desc"], c["flags"], c["kb8"], c["blocked"], c["blocked_r"])
    assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre)
    mt = plvi.ORBmatcher(0.9, True)
    for cut in ("last", "right", "left"):
        d = dict(c)
        if cut == "last":
            for k in ("x3dc", "x3dr", "flags", "last_octave", "last_angle", "mp_desc"):
                d[k] = c[k][:0]
        elif cut == "right":
            d["kps_r"], d["desc_r"], d["blocked_r"] = c["kps_r"][:0], c["desc_r"][:0], c["blocked_r"][:0]
        else:
            d["kps"], d["desc"], d["blocked"] = c["kps"][:0], c["desc"][:0], c["blocked"][:0]
        ne, mle, mre = oracle_lib.search_by_projection_stereo(d, 7.0)
        ng, mlg, mrg = mt.SearchByProjectionStereo(
            util.proj_params(d, 7.0), d["kps"], d["desc"], d["kps_r"], d["desc_r"], d["x3dc"], d["x3dr"],
            d["last_octave"], d["last_angle"], d["mp_desc"], d["flags"], d["kb8"], d["blocked"], d["blocked_r"])
        assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre), cut


@pytest.mark.gpu
def test_stereo_projection_invalid_octave_is_no_candidate():
    """A searched LastFrame point whose octave is outside [0, nlevels) (the reference would index
    mvScaleFactors out of range, ORBmatcher.cc:2029) gets no candidate in either image, in the one-pair
    and the batched entry point alike (the one-pair wrapper runs the batch kernel): the result equals the
    oracle's with those points unflagged."""
    import plvi
    c = util.projection_stereo_case(41)
    rng = np.random.default_rng(5)
    bad = np.nonzero(c["flags"] & 1)[0]
    bad = rng.choice(bad, 40, replace=False)
    d = dict(c)
    d["last_octave"] = c["last_octave"].copy()
    d["last_octave"][bad[:20]] = -1
    d["last_octave"][bad[20:]] = 8
    e = dict(c)
    e["flags"] = c["flags"].copy()
    e["flags"][bad] &= ~np.uint8(1)
    ne, mle, mre = oracle_lib.search_by_projection_stereo(e, 7.0)
    ng, mlg, mrg = plvi.ORBmatcher(0.9, True).SearchByProjectionStereo(
        util.proj_params(d, 7.0), d["kps"], d["desc"], d["kps_r"], d["desc_r"], d["x3dc"], d["x3dr"],
        d["last_octave"], d["last_angle"], d["mp_desc"], d["flags"], d["kb8"], d["blocked"], d["blocked_r"])
    assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre)


@pytest.mark.gpu
def test_stereo_lds_check_counts_static_shared():
    """The LDS capacity checks count the kernels' static __shared__ data (the rotation histogram and
    counters of the two-camera and relocalization SearchByProjection kernels): a configuration whose
    dynamic LDS alone is exactly 160 KB returns PLVI_E_CAPACITY; the local-map stereo kernel has no static
    LDS, so 160 KB launches and 16 B more is refused.  Every pointer is one zeroed device buffer (all
    counts 0), so a launch is harmless."""
    import ctypes
    import plvi
    lib = plvi.load()
    z = plvi.DeviceBuffer(1 << 20)
    z.upload(np.zeros(1 << 20, np.uint8))
    Z = ctypes.c_void_p(z.ptr)
    pp = plvi.ProjParams()
    pp.nlevels = 8
    # proj2: 16*last + 2*((18*cap + 4*3073 + 15) & ~15) + 64 == 163840 at cap 2000, last 4198
    rc = lib.plvi_search_by_projection_stereo_batch(1, ctypes.byref(pp), None, Z, Z, Z, 2000, *([Z] * 6), 2000,
                                                    *([Z] * 10), 4198, Z, Z, Z, None)
    assert rc == plvi.PLVI_E_CAPACITY
    rp = plvi.RelocParams()
    rp.nlevels, rp.orb_dist = 8, 50
    # reloc: 17*cur + 8*kf + 4*3073 + 64 == 163840 at cur 4004, kf 10427
    rc = lib.plvi_search_reloc_batch(1, ctypes.byref(rp), Z, Z, Z, 4004, *([Z] * 10), 10427, Z, Z, None)
    assert rc == plvi.PLVI_E_CAPACITY
    lp = plvi.LocalParams()
    lp.nlevels = 8
    # local2: 16*mp + 2*((17*cap + 4*3073 + 15) & ~15) + 64 == 163840 at cap 2000, mp 4448
    for mp, want in ((4449, plvi.PLVI_E_CAPACITY), (4448, 0)):
        rc = lib.plvi_search_local_stereo_batch(1, ctypes.byref(lp), Z, Z, Z, 2000, *([Z] * 7), 2000, *([Z] * 11),
                                                mp, Z, Z, Z, None)
        assert rc == want, mp
    lib.plvi_device_synchronize()


@pytest.mark.gpu
def test_stereo_projection_batch_device():
    """Several (CurrentFrame, LastFrame) pairs in one plvi_search_by_projection_stereo_batch launch."""
    import ctypes
    import plvi
    lib = plvi.load()
    cases = [util.projection_stereo_case(80 + i, n_left=600 + 50 * i, n_right=550 + 40 * i, n_last=500 + 60 * i)
             for i in range(3)]
    P, cl, cr, lc = len(cases), 800, 700, 700
    kl = np.zeros((P, cl), plvi.KEYPOINT_DTYPE); kr = np.zeros((P, cr), plvi.KEYPOINT_DTYPE)
    dl = np.zeros((P, cl, 32), np.uint8); dr = np.zeros((P, cr, 32), np.uint8)
    bl = np.zeros((P, cl), np.uint8); br = np.zeros((P, cr), np.uint8)
    nl = np.zeros(P, np.int32); nr = np.zeros(P, np.int32); nlast = np.zeros(P, np.int32)
    x3 = np.zeros((P, lc, 3), np.float32); x3r = np.zeros((P, lc, 3), np.float32)
    oc = np.zeros((P, lc), np.int32); an = np.zeros((P, lc), np.float32)
    md = np.zeros((P, lc, 32), np.uint8); lf = np.zeros((P, lc), np.uint8)
    for p, c in enumerate(cases):
        a, b, m = len(c["kps"]), len(c["kps_r"]), len(c["flags"])
        kl[p, :a] = c["kps"]; dl[p, :a] = c["desc"]; bl[p, :a] = c["blocked"]; nl[p] = a
        kr[p, :b] = c["kps_r"]; dr[p, :b] = c["desc_r"]; br[p, :b] = c["blocked_r"]; nr[p] = b
        x3[p, :m] = c["x3dc"]; x3r[p, :m] = c["x3dr"]; oc[p, :m] = c["last_octave"]; an[p, :m] = c["last_angle"]
        md[p, :m] = c["mp_desc"]; lf[p, :m] = c["flags"]; nlast[p] = m
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
    prm = util.proj_params(cases[0], 7.0)
    prm.check_orientation = 1
    kb = np.ascontiguousarray(cases[0]["kb8"], np.float32)
    ml = plvi.DeviceBuffer(P * cl * 4); mr = plvi.DeviceBuffer(P * cr * 4); nmt = plvi.DeviceBuffer(P * 4)
    V = ctypes.c_void_p
    rc = lib.plvi_search_by_projection_stereo_batch(
        P, ctypes.byref(prm), kb.ctypes.data_as(V), V(dkl), V(dev(dl)), V(dnl), cl, V(dev(bl)), V(col.ptr),
        V(cil.ptr), V(dkr), V(dev(dr)), V(dnr), cr, V(dev(br)), V(cor.ptr), V(cir.ptr), V(dev(x3)), V(dev(x3r)),
        V(dev(oc)), V(dev(an)), V(dev(md)), V(dev(lf)), V(dev(nlast)), lc, V(ml.ptr), V(mr.ptr), V(nmt.ptr), None)
    assert rc == 0
    lib.plvi_device_synchronize()
    ML = ml.download(np.zeros((P, cl), np.int32)); MR = mr.download(np.zeros((P, cr), np.int32))
    N = nmt.download(np.zeros(P, np.int32))
    for p, c in enumerate(cases):
        ne, mle, mre = oracle_lib.search_by_projection_stereo(c, 7.0)
        assert N[p] == ne
        np.testing.assert_array_equal(ML[p, :len(mle)], mle)
        np.testing.assert_array_equal(MR[p, :len(mre)], mre)
