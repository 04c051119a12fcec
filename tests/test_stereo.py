"""Rectified stereo of the stereo Frame constructors:
Frame::ComputeStereoMatches (src/Frame.cc:1228-1406) and
Frame::ComputeStereoMatches_Lines (:1408-1492, with lineSegmentOverlapStereo
:1494-1529, filterLineSegmentDisparity :1531-1542, getLineCoords /
LineIterator, LineMatcher::matchGrid).

Parity unpinned: the reference has no tests for these.  The C++ oracle
(oracle/stereo_oracle.cpp) is checked against literal pure-Python
restatements of the cited lines on extractor output of synthetic rectified
pairs (plvi.synth.stereo_pair: two planted disparities), and the HIP path
(host and batched entry points) is compared with the oracle exactly:
mvuRight, mvDepth, matchGrid table, mvDisparity_l, mvDepth_l, mvle_l."""
import math

import numpy as np
import pytest

import oracle_lib
import util
from plvi import synth

f32 = np.float32
MBF, MB = f32(47.90639384423901), f32(0.11)  # EuRoC-like bf and baseline


def _inv(scale):
    return np.array([f32(1.0) / s for s in scale], np.float32)


def _orb_side(img):
    _, kps, desc = oracle_lib.orb_extract(img)
    return kps, desc, oracle_lib.orb_pyramid(img)


def _dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _py_stereo(kL, dL, kR, dR, pyrL, pyrR, scale, inv, mb, mbf):
    """Literal restatement of Frame::ComputeStereoMatches (float32 arithmetic)."""
    N = len(kL)
    ur = np.full(N, -1, np.float32)
    dp = np.full(N, -1, np.float32)
    nRows = pyrL[0].shape[0]
    rows = [[] for _ in range(nRows)]
    for iR in range(len(kR)):
        y = f32(kR["y"][iR])
        sc = f32(scale[kR["octave"][iR]])  # kpY +/- 2*scale, fused in Frame.cc.o
        maxr, minr = int(math.ceil(util.fmaf(2.0, sc, y))), int(math.floor(util.fmaf(-2.0, sc, y)))
        for yi in range(minr, maxr + 1):
            rows[yi].append(iR)
    minD, maxD = f32(0), f32(mbf / mb)
    vdist = []
    for iL in range(N):
        lev, vL, uL = int(kL["octave"][iL]), f32(kL["y"][iL]), f32(kL["x"][iL])
        cand = rows[int(vL)]
        if not cand:
            continue
        minU, maxU = f32(uL - maxD), f32(uL - minD)
        if maxU < 0:
            continue
        best, bestR = 100, 0
        for iR in cand:
            if kR["octave"][iR] < lev - 1 or kR["octave"][iR] > lev + 1:
                continue
            uR = f32(kR["x"][iR])
            if minU <= uR <= maxU:
                d = _dist(dL[iL], dR[iR])
                if d < best:
                    best, bestR = d, iR
        if best >= 75:
            continue
        sf = inv[lev]
        rnd = lambda v: f32(math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5))  # noqa: E731
        suL, svL, suR0 = rnd(f32(uL * sf)), rnd(f32(vL * sf)), rnd(f32(f32(kR["x"][bestR]) * sf))
        w, L = 5, 5
        IL = pyrL[lev][int(svL) - w:int(svL) + w + 1, int(suL) - w:int(suL) + w + 1].astype(np.int32)
        IL = IL - IL[w, w]
        if suR0 < 0 or suR0 + L + w + 1 >= pyrR[lev].shape[1]:
            continue
        dists = []
        for inc in range(-L, L + 1):
            c = int(suR0 + inc - w)
            IR = pyrR[lev][int(svL) - w:int(svL) + w + 1, c:c + 2 * w + 1].astype(np.int32)
            IR = IR - IR[w, w]
            dists.append(f32(np.abs(IL - IR).sum()))
        bi = int(np.argmin(dists))  # first minimum = strict-< scan
        binc = bi - L
        if binc in (-L, L):
            continue
        d1, d2, d3 = dists[bi - 1], dists[bi], dists[bi + 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            delta = f32(f32(d1 - d3) / f32(f32(2.0) * util.fmaf(-2.0, d2, f32(d1 + d3))))
        if delta < -1 or delta > 1:
            continue
        bu = f32(scale[lev] * f32(f32(suR0 + f32(binc)) + delta))
        disp = f32(uL - bu)
        if disp >= minD and disp < maxD:
            if disp <= 0:
                disp, bu = f32(0.01), f32(float(uL) - 0.01)
            dp[iL], ur[iL] = f32(mbf / disp), bu
            vdist.append((int(d2), iL))
    if vdist:
        vdist.sort()
        th = f32(f32(f32(1.5) * f32(1.4)) * f32(vdist[len(vdist) // 2][0]))
        for d, i in reversed(vdist):
            if f32(d) < th:
                break
            ur[i] = dp[i] = -1
    return ur, dp


@pytest.fixture(scope="module")
def pair0():
    L, R, d = synth.stereo_pair(7)
    return _orb_side(L) + _orb_side(R) + (d,)


def test_oracle_stereo_matches_python(pair0):
    kL, dL, pL, kR, dR, pR, _ = pair0
    scale = util.orb_scale_factors()[:8]
    n, ur, dp = oracle_lib.stereo_match(kL, dL, kR, dR, pL, pR, scale, _inv(scale), MB, MBF)
    pur, pdp = _py_stereo(kL, dL, kR, dR, pL, pR, scale, _inv(scale), MB, MBF)
    assert n > 100
    assert np.array_equal(ur, pur) and np.array_equal(dp, pdp)


def test_oracle_stereo_recovers_planted_disparity(pair0):
    kL, dL, pL, kR, dR, pR, (d0, d1) = pair0
    scale = util.orb_scale_factors()[:8]
    n, ur, dp = oracle_lib.stereo_match(kL, dL, kR, dR, pL, pR, scale, _inv(scale), MB, MBF)
    ok = ur >= 0
    disp = kL["x"][ok] - ur[ok]
    exp = np.where(kL["y"][ok] < 240, d0, d1)
    assert np.mean(np.abs(disp - exp) < 1.5) > 0.9
    assert np.allclose(dp[ok], MBF / disp, rtol=1e-6)


def test_oracle_stereo_empty_sides(pair0):
    kL, dL, pL, kR, dR, pR, _ = pair0
    scale = util.orb_scale_factors()[:8]
    n, ur, dp = oracle_lib.stereo_match(kL, dL, kR[:0], dR[:0], pL, pR, scale, _inv(scale), MB, MBF)
    assert n == 0 and (ur == -1).all() and (dp == -1).all()


# ------------------------------------------------------------------ lines
def _py_overlap(spl, epl, spp, epp):
    ov = 1.0
    if abs(epl - spl) > float(f32(0.1)):
        sln, eln, spn, epn = min(spl, epl), max(spl, epl), min(spp, epp), max(spp, epp)
        length = eln - spn
        if epn < sln or spn > eln:
            ov = 0.0
        elif epn > eln and spn < sln:
            ov = eln - sln
        else:
            ov = min(eln, epn) - max(sln, spn)
        ov = ov / length if length > float(f32(0.01)) else 0.0
        ov = min(ov, 1.0) if ov > 1.0 else ov
    return ov


def _py_stereo_lines(klL, dL, klR, dR, W, H, mbf):
    """Restatement of ComputeStereoMatches_Lines around oracle_lib.match_grid."""
    iw, ih = 64 / W, 48 / H
    n1, n2 = len(klL), len(klR)
    g = lambda k, f: k[f].astype(np.float64)  # noqa: E731
    sx, sy, ex, ey = g(klL, "startPointX"), g(klL, "startPointY"), g(klL, "endPointX"), g(klL, "endPointY")
    lines1 = np.stack([(sx * iw).astype(np.int64), (sy * ih).astype(np.int64), (ex * iw).astype(np.int64),
                       (ey * ih).astype(np.int64)], 1).astype(np.int32)
    grid = [[[] for _ in range(48)] for _ in range(64)]
    dirs = np.zeros((n2, 2))
    for i in range(n2):
        k = klR[i]
        vx = float(f32(k["endPointX"] - k["startPointX"])) * iw
        vy = float(f32(k["endPointY"] - k["startPointY"])) * ih
        m = math.sqrt(util.fma(vx, vx, vy * vy))
        dirs[i] = (vx / m, vy / m)
        for (x, y) in util.line_iterator(float(k["startPointX"]) * iw, float(k["startPointY"]) * ih,
                                         float(k["endPointX"]) * iw, float(k["endPointY"]) * ih):
            if 0 <= x < 64 and 0 <= y < 48:
                grid[x][y].append(i)
    _, m12 = oracle_lib.match_grid(lines1, dL, grid, dR, dirs)
    disp = np.full((n1, 2), -1, np.float32)
    dep = np.full((n1, 2), -1, np.float32)
    for i1 in range(n1):
        i2 = m12[i1]
        if i2 < 0:
            continue
        spl0, spl1, epl0, epl1 = sx[i1], sy[i1], ex[i1], ey[i1]
        r = klR[i2]
        spr0, spr1 = float(r["startPointX"]), float(r["startPointY"])
        epr0, epr1 = float(r["endPointX"]), float(r["endPointY"])
        ov = _py_overlap(spl1, epl1, spr1, epr1)
        with np.errstate(divide="ignore", invalid="ignore"):
            spr0 = float(np.float64(util.fma(spr0, spl1 - epr1, epr0 * (spr1 - spl1))) / np.float64(spr1 - epr1))
            spr1 = spl1
            epr0 = float(np.float64(util.fma(spr0, epl1 - epr1, epr0 * (spr1 - epl1))) / np.float64(spr1 - epr1))
            epr1 = epl1
            ds, de = spl0 - spr0, epl0 - epr0
            mn = de if de < ds else ds
            mx = de if ds < de else ds
            if np.float64(mn) / np.float64(mx) < float(f32(0.7)):
                ds = de = -1.0
        th = float(f32(0.1))
        if ds >= 1 and de >= 1 and abs(spl1 - epl1) > th and abs(spr1 - epr1) > th and ov > float(f32(0.75)):
            disp[i1] = (ds, de)
            dep[i1] = (f32(mbf) / f32(ds), f32(mbf) / f32(de))
    return m12, disp, dep


@pytest.fixture(scope="module")
def line_pair0():
    L, R, d = synth.stereo_pair(11)
    kl, dl, _ = oracle_lib.line_extract(L)
    kr, dr, _ = oracle_lib.line_extract(R)
    return kl, dl, kr, dr, d


def test_oracle_stereo_lines_matches_python(line_pair0):
    kl, dl, kr, dr, _ = line_pair0
    n, m, disp, dep, le = oracle_lib.stereo_lines(kl, dl, kr, dr, None, 640, 480, MBF)
    pm, pdisp, pdep = _py_stereo_lines(kl, dl, kr, dr, 640, 480, MBF)
    assert (m >= 0).sum() > 20 and n > 10
    assert np.array_equal(m, pm)
    assert np.array_equal(disp, pdisp) and np.array_equal(dep, pdep)
    a = np.stack([kl["startPointX"], kl["startPointY"], np.ones(len(kl))], 1).astype(np.float64)
    b = np.stack([kl["endPointX"], kl["endPointY"], np.ones(len(kl))], 1).astype(np.float64)
    c = np.cross(a, b)
    c = c / np.sqrt(c[:, 0] ** 2 + c[:, 1] ** 2)[:, None]
    assert np.array_equal(le, c)


def test_oracle_stereo_lines_planted_disparity(line_pair0):
    kl, dl, kr, dr, (d0, d1) = line_pair0
    n, m, disp, dep, le = oracle_lib.stereo_lines(kl, dl, kr, dr, None, 640, 480, MBF)
    ok = disp[:, 0] > 0
    mid = 0.5 * (kl["startPointY"] + kl["endPointY"])
    exp = np.where(mid < 240, d0, d1)
    assert np.mean(np.abs(disp[ok].mean(1) - exp[ok]) < 2.0) > 0.8


def test_oracle_stereo_lines_empty_right(line_pair0):
    kl, dl, kr, dr, _ = line_pair0
    n, m, disp, dep, le = oracle_lib.stereo_lines(kl, dl, kr[:0], dr[:0], None, 640, 480, MBF)
    assert n == 0 and (m == -1).all() and (disp == -1).all() and (le == 0).all()


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 7, 21])
def test_stereo_match_host_matches_oracle(seed):
    import plvi
    L, R, _ = synth.stereo_pair(seed)
    kL, dL, pL = _orb_side(L)
    kR, dR, pR = _orb_side(R)
    scale = util.orb_scale_factors()[:8]
    n, ur, dp = oracle_lib.stereo_match(kL, dL, kR, dR, pL, pR, scale, _inv(scale), MB, MBF)
    g = plvi.ComputeStereoMatches(kL, dL, kR, dR, pL, pR, scale, _inv(scale), MB, MBF)
    assert g[0] == n > 100
    assert np.array_equal(g[1], ur) and np.array_equal(g[2], dp)


@pytest.mark.gpu
def test_stereo_match_host_edge_cases():
    import plvi
    L, R, _ = synth.stereo_pair(5)
    kL, dL, pL = _orb_side(L)
    kR, dR, pR = _orb_side(R)
    scale = util.orb_scale_factors()[:8]
    for (a, b) in [(kL[:0], kR), (kL, kR[:0]), (kL[:1], kR), (kL, kR[:3]), (kL[:40], kR[::7])]:
        ia = np.arange(len(a))
        ib = np.arange(len(b))
        exp = oracle_lib.stereo_match(a, dL[ia], b, dR[ib], pL, pR, scale, _inv(scale), MB, MBF)
        got = plvi.ComputeStereoMatches(a, dL[ia], b, dR[ib], pL, pR, scale, _inv(scale), MB, MBF)
        assert got[0] == exp[0] and np.array_equal(got[1], exp[1]) and np.array_equal(got[2], exp[2])
    # a small mb (large maxD) and a huge mb (maxD < 1 px: almost nothing survives)
    for mb in (f32(0.01), f32(40.0)):
        exp = oracle_lib.stereo_match(kL, dL, kR, dR, pL, pR, scale, _inv(scale), mb, MBF)
        got = plvi.ComputeStereoMatches(kL, dL, kR, dR, pL, pR, scale, _inv(scale), mb, MBF)
        assert got[0] == exp[0] and np.array_equal(got[1], exp[1]) and np.array_equal(got[2], exp[2])


@pytest.mark.gpu
def test_stereo_match_batch_on_extractor_outputs():
    """Two ORB handles (left / right) extract a batch of pairs on the device;
    plvi_stereo_match_batch reads their keypoints, descriptors and pyramids."""
    import plvi
    B = 6
    pairs = [synth.stereo_pair(100 + i) for i in range(B)]
    lib = plvi.load()
    left = plvi.DeviceBuffer(B * 640 * 480)
    right = plvi.DeviceBuffer(B * 640 * 480)
    left.upload(np.stack([p[0] for p in pairs]))
    right.upload(np.stack([p[1] for p in pairs]))
    el = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B)
    er = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B)
    el.extract_batch(left.ptr, B, 640 * 480, 640)
    er.extract_batch(right.ptr, B, 640 * 480, 640)
    lib.plvi_device_synchronize()
    cap = el.kp_cap
    out = plvi.DeviceBuffer(B * cap * 8 + B * 4 + 4)
    ur, dp, ns, err = out.ptr, out.ptr + B * cap * 4, out.ptr + B * cap * 8, out.ptr + B * cap * 8 + B * 4
    out.upload(np.zeros(B * cap * 2 + B + 1, np.int32))
    plvi.stereo_match_batch(el, er, B, MB, MBF, ur, dp, ns, err)
    lib.plvi_device_synchronize()
    assert plvi.download(err, np.zeros(1, np.int32))[0] == 0
    kp, de, co, _, _ = el.outputs()
    kpr, der, cor, _, _ = er.outputs()
    cnt = plvi.download(co, np.zeros(B, np.int32))
    cntr = plvi.download(cor, np.zeros(B, np.int32))
    allk = plvi.download(kp, np.zeros(B * cap, plvi.KEYPOINT_DTYPE)).reshape(B, cap)
    alld = plvi.download(de, np.zeros((B * cap, 32), np.uint8)).reshape(B, cap, 32)
    allkr = plvi.download(kpr, np.zeros(B * cap, plvi.KEYPOINT_DTYPE)).reshape(B, cap)
    alldr = plvi.download(der, np.zeros((B * cap, 32), np.uint8)).reshape(B, cap, 32)
    scale = el.GetScaleFactors()
    inv = el.GetInverseScaleFactors()
    urh = plvi.download(ur, np.zeros((B, cap), np.float32))
    dph = plvi.download(dp, np.zeros((B, cap), np.float32))
    nsh = plvi.download(ns, np.zeros(B, np.int32))
    for f in range(B):
        pL = [el.pyramid_level(l, f) for l in range(8)]
        pR = [er.pyramid_level(l, f) for l in range(8)]
        n, eu, ed = oracle_lib.stereo_match(allk[f, :cnt[f]], alld[f, :cnt[f]], allkr[f, :cntr[f]],
                                            alldr[f, :cntr[f]], pL, pR, scale, inv, MB, MBF)
        assert nsh[f] == n > 100
        assert np.array_equal(urh[f, :cnt[f]], eu) and np.array_equal(dph[f, :cnt[f]], ed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_stereo_lines_gcc10_order_matches_oracle(seed):
    """ComputeStereoMatches_Lines with the shipped candidate order
    (range_hint=1, GCC <= 10 unordered_set range insert)."""
    import plvi
    L, R, _ = synth.stereo_pair(seed)
    kl, dl, _ = oracle_lib.line_extract(L)
    kr, dr, _ = oracle_lib.line_extract(R)
    exp = oracle_lib.stereo_lines(kl, dl, kr, dr, None, 640, 480, MBF, range_hint=1)
    got = plvi.ComputeStereoMatches_Lines(kl, dl, kr, dr, None, 640, 480, MBF, range_hint=1)
    assert got[0] == exp[0] > 10
    for g, e in zip(got[1:], exp[1:]):
        assert np.array_equal(g, e)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_stereo_lines_host_matches_oracle(seed):
    import plvi
    L, R, _ = synth.stereo_pair(seed)
    kl, dl, _ = oracle_lib.line_extract(L)
    kr, dr, _ = oracle_lib.line_extract(R)
    un = kl.copy()
    un["startPointX"] += f32(0.25)  # mvKeysUn_Line distinct from mvKeys_Line
    exp = oracle_lib.stereo_lines(kl, dl, kr, dr, un, 640, 480, MBF)
    got = plvi.ComputeStereoMatches_Lines(kl, dl, kr, dr, un, 640, 480, MBF, range_hint=0)
    assert got[0] == exp[0] > 10
    for g, e in zip(got[1:], exp[1:]):
        assert np.array_equal(g, e)
    # empty right side: no matches, mvle_l left at zero
    got = plvi.ComputeStereoMatches_Lines(kl, dl, kr[:0], dr[:0], un, 640, 480, MBF, range_hint=0)
    assert got[0] == 0 and (got[1] == -1).all() and (got[4] == 0).all()


@pytest.mark.gpu
def test_stereo_lines_batch_on_extractor_outputs():
    import plvi
    B = 4
    pairs = [synth.stereo_pair(200 + i) for i in range(B)]
    lib = plvi.load()
    left = plvi.DeviceBuffer(B * 640 * 480)
    right = plvi.DeviceBuffer(B * 640 * 480)
    left.upload(np.stack([p[0] for p in pairs]))
    right.upload(np.stack([p[1] for p in pairs]))
    xl = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
    xr = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
    xl.extract_batch(left.ptr, B, 640 * 480, 640)
    xr.extract_batch(right.ptr, B, 640 * 480, 640)
    lib.plvi_device_synchronize()
    kl, dl, _, cl, cap = xl.outputs()
    kr, dr, _, cr, capr = xr.outputs()
    idx_cap = 32768
    sb = plvi.stereo_lines_scratch_bytes(B, cap, capr, idx_cap)
    scratch = plvi.DeviceBuffer(sb)
    o = plvi.DeviceBuffer(B * cap * (4 + 8 + 8 + 24) + B * 4 + 4)
    m12 = o.ptr
    disp = m12 + B * cap * 4
    dep = disp + B * cap * 8
    le = dep + B * cap * 8
    ns = le + B * cap * 24
    err = ns + B * 4
    o.upload(np.zeros(o.nbytes, np.uint8))
    plvi.stereo_lines_batch(B, kl, dl, cl, cap, kr, dr, cr, capr, None, 640, 480, MBF, 0, idx_cap,
                            scratch.ptr, sb, m12, disp, dep, le, ns, err)
    lib.plvi_device_synchronize()
    assert plvi.download(err, np.zeros(1, np.int32))[0] == 0
    nl = plvi.download(cl, np.zeros(B, np.int32))
    nr = plvi.download(cr, np.zeros(B, np.int32))
    KL = plvi.download(kl, np.zeros(B * cap, plvi.KEYLINE_DTYPE)).reshape(B, cap)
    DL = plvi.download(dl, np.zeros((B * cap, 32), np.uint8)).reshape(B, cap, 32)
    KR = plvi.download(kr, np.zeros(B * capr, plvi.KEYLINE_DTYPE)).reshape(B, capr)
    DR = plvi.download(dr, np.zeros((B * capr, 32), np.uint8)).reshape(B, capr, 32)
    m12h = plvi.download(m12, np.zeros((B, cap), np.int32))
    disph = plvi.download(disp, np.zeros((B, cap, 2), np.float32))
    deph = plvi.download(dep, np.zeros((B, cap, 2), np.float32))
    leh = plvi.download(le, np.zeros((B, cap, 3), np.float64))
    nsh = plvi.download(ns, np.zeros(B, np.int32))
    for f in range(B):
        a, b = KL[f, :nl[f]], KR[f, :nr[f]]
        n, m, d, z, l_ = oracle_lib.stereo_lines(a, DL[f, :nl[f]], b, DR[f, :nr[f]], None, 640, 480, MBF)
        assert nsh[f] == n > 5
        assert np.array_equal(m12h[f, :nl[f]], m)
        assert np.array_equal(disph[f, :nl[f]], d) and np.array_equal(deph[f, :nl[f]], z)
        assert np.array_equal(leh[f, :nl[f]], l_)


@pytest.mark.gpu
def test_stereo_frame_schedule_then_stereo_matching():
    """The stereo-line Frame (src/Frame.cc:200-249) as one call: ORB and lines
    of the left and right images as two concurrent frame schedules
    (plvi_stereo_frame_extract_batch), then ComputeStereoMatches and
    ComputeStereoMatches_Lines on the same stream.  Each side equals its own
    single-schedule extraction bit for bit, a left and a right frame equal
    the oracle, and the stereo tables equal the oracle's on every pair."""
    import torch
    import plvi
    B = 4
    pairs = [synth.stereo_pair(300 + i) for i in range(B)]
    lib = plvi.load()
    L = np.stack([p[0] for p in pairs])
    R = np.stack([p[1] for p in pairs])
    bl, br = plvi.DeviceBuffer(L.nbytes), plvi.DeviceBuffer(R.nbytes)
    bl.upload(L)
    br.upload(R)
    mk = lambda: (plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B),  # noqa: E731
                  plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B))
    (ol_, ll_), (or_, lr_) = mk(), mk()
    s = torch.cuda.Stream()
    st = s.cuda_stream
    plvi.stereo_frame_extract_batch(ol_, or_, ll_, lr_, bl.ptr, br.ptr, B, 640 * 480, 640, stream=st)
    cap = ol_.kp_cap
    out = plvi.DeviceBuffer(B * cap * 8 + B * 4 + 4)
    ur, dp, ns, err = out.ptr, out.ptr + B * cap * 4, out.ptr + B * cap * 8, out.ptr + B * cap * 8 + B * 4
    out.upload(np.zeros(B * cap * 2 + B + 1, np.int32))
    plvi.stereo_match_batch(ol_, or_, B, MB, MBF, ur, dp, ns, err, stream=st)
    kl, dl, _, cl, lcap = ll_.outputs()
    kr, dr, _, cr, lcapr = lr_.outputs()
    idx_cap = 32768
    sb = plvi.stereo_lines_scratch_bytes(B, lcap, lcapr, idx_cap)
    scratch = plvi.DeviceBuffer(sb)
    o = plvi.DeviceBuffer(B * lcap * (4 + 8 + 8 + 24) + B * 4 + 4)
    m12 = o.ptr
    disp, dep = m12 + B * lcap * 4, m12 + B * lcap * 12
    le, lns = m12 + B * lcap * 20, m12 + B * lcap * 44
    lerr = lns + B * 4
    o.upload(np.zeros(o.nbytes, np.uint8))
    plvi.stereo_lines_batch(B, kl, dl, cl, lcap, kr, dr, cr, lcapr, None, 640, 480, MBF, 0, idx_cap, scratch.ptr, sb,
                            m12, disp, dep, le, lns, lerr, stream=st)
    torch.cuda.synchronize()
    assert plvi.download(err, np.zeros(1, np.int32))[0] == 0 and plvi.download(lerr, np.zeros(1, np.int32))[0] == 0
    assert ol_.errors() == 0 and or_.errors() == 0 and ll_.errors() == 0 and lr_.errors() == 0

    def tabs(orb, lx):
        kp, de, co, _, c = orb.outputs()
        k2, d2, _, c2, cc = lx.outputs()
        n = plvi.download(co, np.zeros(B, np.int32))
        m = plvi.download(c2, np.zeros(B, np.int32))
        K = plvi.download(kp, np.zeros(B * c, plvi.KEYPOINT_DTYPE)).reshape(B, c)
        D = plvi.download(de, np.zeros((B * c, 32), np.uint8)).reshape(B, c, 32)
        KL = plvi.download(k2, np.zeros(B * cc, plvi.KEYLINE_DTYPE)).reshape(B, cc)
        DL = plvi.download(d2, np.zeros((B * cc, 32), np.uint8)).reshape(B, cc, 32)
        return [(K[f, :n[f]], D[f, :n[f]], KL[f, :m[f]], DL[f, :m[f]]) for f in range(B)]
    sides = tabs(ol_, ll_), tabs(or_, lr_)
    # each side equals its own single-side frame schedule
    for img_buf, side in ((bl, sides[0]), (br, sides[1])):
        o2, l2 = mk()
        plvi.frame_extract_batch(o2, l2, img_buf.ptr, B, 640 * 480, 640)
        lib.plvi_device_synchronize()
        for a, b in zip(side, tabs(o2, l2)):
            assert all(x.tobytes() == y.tobytes() for x, y in zip(a, b))
    # left frame 0 and right frame B-1 against the oracle
    for img, t in ((L[0], sides[0][0]), (R[B - 1], sides[1][B - 1])):
        _, ek, ed = oracle_lib.orb_extract(img)
        assert t[0].tobytes() == ek.astype(plvi.KEYPOINT_DTYPE).tobytes() and np.array_equal(t[1], ed)
        ekl, eld, _ = oracle_lib.line_extract(img)
        assert t[2].tobytes() == ekl.astype(plvi.KEYLINE_DTYPE).tobytes() and np.array_equal(t[3], eld)
    # stereo tables
    scale, inv = ol_.GetScaleFactors(), ol_.GetInverseScaleFactors()
    urh = plvi.download(ur, np.zeros((B, cap), np.float32))
    dph = plvi.download(dp, np.zeros((B, cap), np.float32))
    nsh = plvi.download(ns, np.zeros(B, np.int32))
    m12h = plvi.download(m12, np.zeros((B, lcap), np.int32))
    lnsh = plvi.download(lns, np.zeros(B, np.int32))
    for f in range(B):
        (k, d, a, da), (kr_, dr_, b, db) = sides[0][f], sides[1][f]
        pL = [ol_.pyramid_level(lv, f) for lv in range(8)]
        pR = [or_.pyramid_level(lv, f) for lv in range(8)]
        n, eu, ed = oracle_lib.stereo_match(k, d, kr_, dr_, pL, pR, scale, inv, MB, MBF)
        assert nsh[f] == n > 100
        assert np.array_equal(urh[f, :len(k)], eu) and np.array_equal(dph[f, :len(k)], ed)
        n2, m, _, _, _ = oracle_lib.stereo_lines(a, da, b, db, None, 640, 480, MBF)
        assert lnsh[f] == n2 > 5 and np.array_equal(m12h[f, :len(a)], m)
