"""Known-answer tests that pin the CPU oracle's OpenCV/libm primitives
(SURVEY.md Appendix A).  No reference test exists for them, so these are the
pins: closed forms checked against independent restatements, constants
against the values the reference's own parameters imply."""
import numpy as np
import pytest

import oracle_lib as ol
from plvi import synth


def test_gaussian_fixed_point_taps_error_diffusion():
    assert list(ol.gaussian_taps(7, 2.0)) == [18, 34, 48, 56, 48, 34, 18]   # ORB 7x7 sigma 2
    assert list(ol.gaussian_taps(5, 1.0)) == [14, 62, 104, 62, 14]          # LBD 5x5 sigma 1
    assert ol.gaussian_taps(7, 2.0).sum() == 256


def test_gaussian_f64_kernel_lsd():
    k = ol.gaussian_kernel_f64(7, 0.75)
    assert abs(k.sum() - 1.0) < 1e-15
    x = np.arange(-3, 4)
    ref = np.exp(-x * x / (2 * 0.75 ** 2))
    np.testing.assert_allclose(k, ref / ref.sum(), rtol=1e-14)


def _corner_score_opencv_loop(d, threshold):
    # cornerScore<16> scalar loop form (OpenCV 4.2 features2d/src/fast_score.cpp)
    d = list(d) + list(d[:9])
    a0 = threshold
    for k in range(0, 16, 2):
        a = min(d[k + 1], d[k + 2], d[k + 3])
        if a <= a0:
            continue
        a = min(a, d[k + 4], d[k + 5], d[k + 6], d[k + 7], d[k + 8])
        a0 = max(a0, min(a, d[k]))
        a0 = max(a0, min(a, d[k + 9]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = max(d[k + 1], d[k + 2], d[k + 3], d[k + 4], d[k + 5])
        if b >= b0:
            continue
        b = max(b, d[k + 6], d[k + 7], d[k + 8])
        b0 = min(b0, max(b, d[k]))
        b0 = min(b0, max(b, d[k + 9]))
    return -b0 - 1


CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _is_corner(d, t):
    dd = list(d) * 2
    for s in range(16):
        arc = dd[s:s + 9]
        if all(v > t for v in arc) or all(-v > t for v in arc):
            return True
    return False


def test_fast_score_closed_form_matches_opencv_loop():
    lib = ol.load()
    rng = np.random.default_rng(7)
    checked = 0
    for trial in range(20000):
        patch = rng.integers(0, 256, size=(7, 7), dtype=np.uint8)
        if trial % 2:
            # planted arcs make corners common
            v = int(patch[3, 3])
            s = rng.integers(0, 16)
            for i in range(rng.integers(8, 13)):
                dx, dy = CIRCLE[(s + i) % 16]
                patch[3 + dy, 3 + dx] = np.clip(v + rng.choice([-1, 1]) * rng.integers(10, 90), 0, 255)
        patch = np.ascontiguousarray(patch)
        S = lib.oracle_fast_score(ctypes_ptr(patch, 3 * 7 + 3), 7)
        v = int(patch[3, 3])
        d = [v - int(patch[3 + dy, 3 + dx]) for dx, dy in CIRCLE]
        for t in (7, 20):
            corner = _is_corner(d, t)
            assert corner == (S > t)
            if corner:
                assert _corner_score_opencv_loop(d, t) == S - 1
                checked += 1
    assert checked > 1000


def ctypes_ptr(a, offset):
    import ctypes
    return ctypes.c_void_p(a.ctypes.data + offset)


def test_fast_atan2_constants_and_quadrants():
    lib = ol.load()
    assert lib.oracle_fast_atan2(0.0, 1.0) == 0.0
    assert abs(lib.oracle_fast_atan2(1.0, 0.0) - 90.0) < 1e-3
    assert abs(lib.oracle_fast_atan2(0.0, -1.0) - 180.0) < 1e-3
    assert abs(lib.oracle_fast_atan2(-1.0, 0.0) - 270.0) < 1e-3
    rng = np.random.default_rng(1)
    for y, x in rng.normal(size=(2000, 2)) * 100:
        a = lib.oracle_fast_atan2(float(y), float(x))
        ref = np.degrees(np.arctan2(np.float32(y), np.float32(x))) % 360
        assert abs(((a - ref) + 180) % 360 - 180) < 0.02   # OpenCV documents ~0.3 deg worst case


def test_resize_half_is_area_fast_path():
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, size=(240, 322), dtype=np.uint8)   # 161 = 20*8 + 1 -> scalar tail column
    out = ol.resize(src, 161, 120)
    s = src.astype(np.int32)
    tot = s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2]
    simd = (tot + 2) >> 2
    tail = np.rint(tot.astype(np.float32) * np.float32(0.25)).astype(np.int32)   # cvRound half-even
    exp = simd.copy()
    exp[:, 160:] = tail[:, 160:]
    assert np.array_equal(out, exp.astype(np.uint8))


def test_resize_bilinear_fixed_point_formula():
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, size=(480, 640), dtype=np.uint8)
    dw, dh = 533, 400
    out = ol.resize(src, dw, dh)
    sx_scale = 1.0 / (dw / 640.0)
    sy_scale = 1.0 / (dh / 480.0)
    s = src.astype(np.int64)
    for dy in (0, 1, 199, 399):
        fy = np.float32((dy + 0.5) * sy_scale - 0.5)
        sy = int(np.floor(fy)); fy = np.float32(fy - np.float32(sy))
        b0 = int(np.rint(np.float32(1.0 - fy) * np.float32(2048))); b1 = int(np.rint(fy * np.float32(2048)))
        for dx in (0, 1, 266, 532):
            fx = np.float32((dx + 0.5) * sx_scale - 0.5)
            sx = int(np.floor(fx)); fx = np.float32(fx - np.float32(sx))
            a0 = int(np.rint(np.float32(1.0 - fx) * np.float32(2048))); a1 = int(np.rint(fx * np.float32(2048)))
            H0 = s[sy, sx] * a0 + s[sy, sx + 1] * a1
            H1 = s[sy + 1, sx] * a0 + s[sy + 1, sx + 1] * a1
            v = (((b0 * (H0 >> 4)) >> 16) + ((b1 * (H1 >> 4)) >> 16) + 2) >> 2
            assert out[dy, dx] == v


def test_orb_constructor_tables():
    import ctypes
    lib = ol.load()
    scale = (ctypes.c_float * 8)(); per = (ctypes.c_int * 8)(); um = (ctypes.c_int * 16)()
    lib.oracle_orb_params(1000, 1.2, 8, scale, per, um)
    assert list(per) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(um) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    np.testing.assert_array_equal(np.float32(list(scale)), np.float32(
        [1.0, 1.2000000477, 1.4400000572, 1.7280001640, 2.0736002922, 2.4883203506, 2.9859845638, 3.5831816196]))
    lib.oracle_orb_params(5000, 1.2, 8, scale, per, um)
    assert list(per) == [1086, 905, 754, 628, 524, 436, 364, 303]


def test_oracle_orb_is_deterministic_and_bounded():
    img = synth.frame(11)
    m1, k1, d1 = ol.orb_extract(img)
    m2, k2, d2 = ol.orb_extract(img)
    assert m1 == m2 and np.array_equal(k1, k2) and np.array_equal(d1, d2)
    quota = [217, 181, 151, 126, 105, 87, 73, 60]
    for l in range(8):
        assert (k1["octave"] == l).sum() <= quota[l] + 2
    assert len(k1) > 900
    assert m1 == len(k1)  # vLappingArea {0,0}: nothing in the stereo slots


def test_oracle_lapping_area_reverses_order():
    img = synth.frame(12)
    m, k, d = ol.orb_extract(img)
    m2, k2, d2 = ol.orb_extract(img, lap=(0, 1000))
    assert m2 == 0
    assert np.array_equal(k2[::-1], k) and np.array_equal(d2[::-1], d)


def test_is_aligned_float_prefilter_matches_double():
    """lsd_grow_kernel's is_aligned_fast: the float |T - D| decision outside a
    1e-3 degree margin around prec / 360 - prec equals lsd.cpp's double
    isAligned(a = D*DEG_TO_RADS, theta = T*DEG_TO_RADS, prec) (:1136-1152)."""
    rng = np.random.default_rng(5)
    f32, f64 = np.float32, np.float64
    d2r = np.pi / 180
    prec = np.pi * 22.5 / 180
    pdeg = f32(prec / d2r)
    n = 400000
    T = rng.uniform(0, 360, n).astype(f32)
    D = rng.uniform(0, 360, n).astype(f32)
    # adversarial: differences near 22.5, 337.5, 270 and tiny angles
    k = n // 4
    off = rng.choice([22.5, -22.5, 337.5, -337.5, 270.0, -270.0], k) + rng.normal(0, 2e-3, k)
    D[:k] = rng.uniform(0, 360, k).astype(f32)
    T[:k] = np.clip(D[:k].astype(f64) + off, 0, 359.9999).astype(f32)
    T[k:k + 1000] = rng.uniform(0, 1e-6, 1000).astype(f32)
    a = D.astype(f64) * d2r
    th = T.astype(f64) * d2r
    dd = np.abs(th - a)
    n_theta = np.where(dd > 3 * np.pi / 2, np.abs(dd - 2 * np.pi), dd)
    exact = n_theta <= prec
    df = np.abs(T - D).astype(f32)
    near = (np.abs(df - pdeg) < f32(1e-3)) | (np.abs(df - (f32(360) - pdeg)) < f32(1e-3))
    fast = (df <= pdeg) | (df >= f32(360) - pdeg)
    assert near.sum() > 100  # the margin is exercised
    assert np.array_equal(fast[~near], exact[~near])


def test_octree_tie_order_diagnostic():
    """SURVEY §8c diagnostic (B.1): the reference breaks DistributeOctTree's
    equal-size ties by heap address; other tie orders replace a few percent of
    the keypoints (tools/octree_tie_diag.py), and mode 0 (creation order, the
    canonical rule of the oracle and the HIP path) is restored afterwards."""
    import sys
    sys.path.insert(0, str(ol.ROOT / "tools"))
    import octree_tie_diag
    img = synth.frame(3)
    before = ol.orb_extract(img)[1]
    nf, out = octree_tie_diag.run(2)
    assert nf >= 2 and set(out) == {"reverse", "random"}
    for lv, fr, kp in out.values():
        assert 0.0 < kp < 0.2  # some, but few, keypoints depend on the tie order
    after = ol.orb_extract(img)[1]
    assert before.tobytes() == after.tobytes()
