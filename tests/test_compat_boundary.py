"""OpenCV-semantics switches (PLVI_COMPAT_*) and the
drop-in boundary fixes of round 2.

CPU (oracle): the switch settings reproduce the alternatives SURVEY A.1 /
A.4 / A.6 name, and each switch changes something on a real input (so the
GPU parity tests below are not vacuous).

GPU: for every switch setting the HIP path equals the oracle run under the
same setting, bit for bit; handles accept any frame size (operator()
semantics); per-frame batch error flags; matchNNR / match keep the caller's
existing matches_12 entries like the reference's std::vector resize."""
import math

import numpy as np
import pytest

import oracle_lib as ol
from plvi import synth
from util import real_frames

SIGMA_LSD = 0.6 / float(np.float32(0.8))


def _taps(n, sigma):
    t = np.zeros(n, np.int32)
    ol.load().oracle_gaussian_taps_u8(n, sigma, ol._p(t))
    return t.tolist()


def test_compat_taps_kat():
    # A.4: error diffusion (default) vs plain rounding (sum 257)
    assert _taps(7, 2.0) == [18, 34, 48, 56, 48, 34, 18]
    assert _taps(5, 1.0) == [14, 62, 104, 62, 14]
    with ol.compat(1):
        assert _taps(7, 2.0) == [18, 34, 49, 55, 49, 34, 18]
        assert _taps(5, 1.0) == [14, 63, 103, 63, 14]


def test_compat_cv_exp_table():
    # exp64f restatement: exact at 0, within ~1e-14 relative of glibc elsewhere
    assert ol.cv_exp_table(0.0) == 1.0
    rng = np.random.default_rng(0)
    for x in rng.uniform(-30, 5, 2000):
        e, c = math.exp(x), ol.cv_exp_table(x)
        assert abs(e - c) <= 2e-14 * e, (x, e, c)
    # A.6: the two exps give different f64 LSD kernels at the config's sigma
    k0, k4 = np.zeros(7), np.zeros(7)
    ol.load().oracle_gaussian_kernel_f64(7, SIGMA_LSD, ol._p(k0))
    with ol.compat(4):
        ol.load().oracle_gaussian_kernel_f64(7, SIGMA_LSD, ol._p(k4))
    assert not np.array_equal(k0, k4)
    assert np.allclose(k0, k4, rtol=1e-15, atol=0)


def test_compat_resize_generic_changes_pyramid():
    img = synth.frame(5)
    a = ol.orb_stage(img, 3)["pyr"]
    with ol.compat(2):
        b = ol.orb_stage(img, 3)["pyr"]
    assert a.shape == b.shape and (a != b).any()
    assert np.abs(a.astype(int) - b.astype(int)).max() <= 3  # level 3 = three chained resizes


# ------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


def _same_orb(got, exp, tag):
    from test_orb_gpu import _assert_same
    _assert_same(got, exp, tag)


def _same_lines(got, exp, tag):
    from test_lines_gpu import _assert_same
    _assert_same(got, exp, tag)


@gpu
@pytest.mark.parametrize("bits", [1, 2, 3])
def test_orb_compat_parity(plvi_lib, bits):
    import plvi
    ext = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, compat=bits)
    imgs = {"synth0": synth.frame(0), "rgb1_gray": real_frames()["rgb1_gray"]}
    with ol.compat(bits):
        for k, img in imgs.items():
            _same_orb(ext(img), ol.orb_extract(img), f"compat{bits} {k}")


@gpu
@pytest.mark.parametrize("bits", [1, 4, 5])
def test_lines_compat_parity(plvi_lib, bits):
    import plvi
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, compat=bits)
    imgs = {"synth1": synth.frame(1), "rgb1_gray": real_frames()["rgb1_gray"]}
    with ol.compat(bits):
        for k, img in imgs.items():
            _same_lines(lx(img), ol.line_extract(img), f"compat{bits} {k}")


@gpu
def test_frame_batch_compat_all(plvi_lib):
    """The frame schedule (ORB || lines) under every switch at once."""
    import plvi
    bits = 7
    B = 2
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B, compat=bits)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B, compat=bits)
    frames = synth.batch(B, seed0=300)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    plvi.frame_extract_batch(orb, lx, buf.ptr, B, 640 * 480, 640, (0, 0))
    plvi.load().plvi_device_synchronize()
    kp_p, de_p, co_p, mo_p, cap = orb.outputs()
    cnt = plvi.download(co_p, np.zeros(B, np.int32))
    mono = plvi.download(mo_p, np.zeros(B, np.int32))
    kps = plvi.download(kp_p, np.zeros(B * cap, plvi.KEYPOINT_DTYPE))
    desc = plvi.download(de_p, np.zeros((B * cap, 32), np.uint8))
    klp, dep, fnp, lcop, lcap = lx.outputs()
    lcnt = plvi.download(lcop, np.zeros(B, np.int32))
    kl = plvi.download(klp, np.zeros(B * lcap, plvi.KEYLINE_DTYPE))
    lde = plvi.download(dep, np.zeros((B * lcap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((B * lcap, 3), np.float64))
    assert orb.errors() == 0 and lx.errors() == 0
    with ol.compat(bits):
        for f in range(B):
            s = slice(f * cap, f * cap + cnt[f])
            _same_orb((int(mono[f]), kps[s], desc[s]), ol.orb_extract(frames[f]), f"frame{f} orb")
            s = slice(f * lcap, f * lcap + lcnt[f])
            _same_lines((kl[s], lde[s], fn[s]), ol.line_extract(frames[f]), f"frame{f} lines")


@gpu
def test_handles_accept_any_frame_size(plvi_lib):
    """ORBextractor / Lineextractor operator() take any image size
    (ORBextractor.cc:1152-1160, LineExtractor.cc:45): a handle created for
    640x480 re-plans for 752x480 and back."""
    import plvi
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480)
    fr = real_frames()
    for img in (fr["euroc1"], fr["rgb1_gray"], fr["euroc2"], synth.frame(9, 320, 240)):
        _same_orb(orb(img), ol.orb_extract(img), f"orb {img.shape}")
        _same_lines(lx(img), ol.line_extract(img), f"lines {img.shape}")
        assert orb.pyramid_level(0).shape == img.shape


@gpu
def test_batch_error_flags_read_and_clear(plvi_lib):
    import plvi
    B = 3
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
    frames = synth.batch(B, seed0=7)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    plvi.frame_extract_batch(orb, lx, buf.ptr, B, 640 * 480, 640, (0, 0))
    fo, fl = orb.errors(per_frame=True), lx.errors(per_frame=True)
    assert fo.shape == (B,) and fl.shape == (B,) and not fo.any() and not fl.any()
    assert orb.errors() == 0 and lx.errors() == 0


@gpu
def test_match_nnr_keeps_existing_entries(plvi_lib):
    """matches_12.resize(rows, -1) keeps a caller's earlier entries
    (LineMatcher.cpp:44): only accepted matches overwrite them, and match()
    mutual-checks kept entries too (LineMatcher.cpp:101-106)."""
    import plvi
    rng = np.random.default_rng(5)
    d2 = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    bits = np.unpackbits(d2[:30], axis=1)
    bits ^= (rng.random(bits.shape) < 0.06).astype(np.uint8)
    d1 = np.concatenate([np.packbits(bits, axis=1), rng.integers(0, 256, (20, 32), dtype=np.uint8)])
    for prev in (None, np.arange(10, dtype=np.int32), np.full(50, 7, np.int32), np.full(80, 3, np.int32),
                 rng.integers(-1, 40, 50).astype(np.int32)):
        for fn_g, fn_o in ((plvi.LineMatcher.matchNNR, ol.match_nnr), (plvi.LineMatcher.match, ol.match)):
            ng, mg = fn_g(d1, d2, 0.9, prev)
            ne, me = fn_o(d1, d2, 0.9, prev)
            assert ng == ne and np.array_equal(mg, me), (fn_g.__name__, None if prev is None else prev[:5])
    # a kept entry beyond desc2's rows is undefined in match(): refused
    stale = np.full(50, 45, np.int32)
    with pytest.raises(plvi.PlviError):
        plvi.LineMatcher.match(d1, d2, 0.9, stale)
    assert ol.match(d1, d2, 0.9, stale)[0] == -2
