"""LSD plane parity (lsd.cpp:412-584): the prep kernel's angle and modgrad
planes equal the oracle's flsd planes bit for bit, on both octaves; the
per-pixel cos/sin pairs equal glibc's cosf/sinf of float(angle)."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import real_frames

pytestmark = pytest.mark.gpu

D2R = np.pi / 180


def _frames():
    fr = real_frames()
    return [("synth0", synth.frame(0)), ("synth7", synth.frame(7)), ("rgb1_gray", fr["rgb1_gray"]),
            ("euroc1", fr["euroc1"])]


def _check_vs_oracle(lx, img, tag, scale=0.8):
    lx(img)
    for lvl in range(2):
        deg, mg, _ = lx.debug_planes(lvl)
        src = img if lvl == 0 else lx.pyramid_level(1)
        _, ang, mge = ol.lsd_planes(src, scale)
        assert deg.shape == ang.shape, tag
        nd = ang == -1024.0
        assert np.array_equal(deg == -1024.0, nd), f"{tag} L{lvl}: NOTDEF sets differ"
        a = deg.astype(np.float64) * D2R
        bad = np.flatnonzero((a.view(np.uint64) != ang.view(np.uint64)) & ~nd)
        assert bad.size == 0, f"{tag} L{lvl}: angles differ at {bad[:8]}"
        bad = np.flatnonzero(mg.view(np.uint64) != mge.view(np.uint64))
        assert bad.size == 0, f"{tag} L{lvl}: modgrad differs at {bad[:8]} {mg.ravel()[bad[:4]]} {mge.ravel()[bad[:4]]}"


@pytest.mark.parametrize("k", range(4))
def test_lsd_planes_match_oracle(plvi_lib, k):
    tag, img = _frames()[k]
    h, w = img.shape
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, w, h)
    _check_vs_oracle(lx, img, tag)


def test_lsd_pixel_cos_sin_match_glibc(plvi_lib):
    """region_grow's per-pixel cos/sin(float(angle)) (lsd.cpp:678-679), stored
    by the prep kernel for defined pixels, equal this host's glibc cosf/sinf."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for fn in (libm.cosf, libm.sinf):
        fn.restype, fn.argtypes = ctypes.c_float, [ctypes.c_float]
    img = synth.frame(3)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480)
    lx(img)
    for lvl in range(2):
        deg, _, cs = lx.debug_planes(lvl)
        df = deg != -1024.0
        x = (deg[df].astype(np.float64) * D2R).astype(np.float32)
        c = np.array([libm.cosf(float(v)) for v in x], np.float32)
        s = np.array([libm.sinf(float(v)) for v in x], np.float32)
        assert np.array_equal(cs[df][:, 0].view(np.uint32), c.view(np.uint32)), f"L{lvl} cos"
        assert np.array_equal(cs[df][:, 1].view(np.uint32), s.view(np.uint32)), f"L{lvl} sin"


def test_lines_lsd_scale_one(plvi_lib):
    """SCALE = 1: flsd skips the blur / resize (lsd.cpp:460-463)."""
    img = synth.frame(5)
    lx = plvi.Lineextractor(200, 0, 1.0, 2, 2.0, 0, 640, 480)
    lx(img)
    deg, mg, _ = lx.debug_planes(0)
    _, ang, mge = ol.lsd_planes(img, 1.0)
    assert np.array_equal(mg.view(np.uint64), mge.view(np.uint64))
    kg, dg, fg = lx(img)
    ke, de, fe = ol.line_extract(img, lsd_scale=1.0)
    assert len(kg) == len(ke) and kg.tobytes() == ke.tobytes() and np.array_equal(dg, de)
