"""Multi-wave region growing (lsd_grow_mw_kernel, small batches): several
regions of one frame grow concurrently and commit in raster seed order after
validation (lsd.cpp:476-533, 635-686).  Parity: the lines equal the oracle's
and the sequential kernel's bit for bit; the counters show the speculative
path, the regrow path and the walker's exact path all ran."""
import ctypes

import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import real_frames, structured_frames

pytestmark = pytest.mark.gpu


def _tables(lx, n):
    klp, dep, fnp, cop, cap = lx.outputs()
    cnt = plvi.download(cop, np.zeros(n, np.int32))
    kl = plvi.download(klp, np.zeros(n * cap, plvi.KEYLINE_DTYPE))
    de = plvi.download(dep, np.zeros((n * cap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((n * cap, 3), np.float64))
    return [(kl[f * cap:f * cap + cnt[f]], de[f * cap:f * cap + cnt[f]], fn[f * cap:f * cap + cnt[f]])
            for f in range(n)]


def _same(a, b):
    return a[0].tobytes() == b[0].tobytes() and np.array_equal(a[1], b[1]) and a[2].tobytes() == b[2].tobytes()


def _run(monkeypatch, frames, mw, stats=False):
    monkeypatch.setenv("PLVI_GROW_MW", str(mw))
    n, h, w = frames.shape
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, w, h, max_batch=n)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    st = None
    lib = plvi.load()
    if stats:
        st = plvi.DeviceBuffer(n * 2 * 16 * 4)
        st.upload(np.zeros(n * 2 * 16, np.int32))
        lib.plvi_lines_debug_mw_stats(lx._h, ctypes.c_void_p(st.ptr))
    lx.extract_batch(buf.ptr, n, w * h, w)
    lib.plvi_device_synchronize()
    assert lx.errors() == 0
    out = _tables(lx, n)
    if stats:
        lib.plvi_lines_debug_mw_stats(lx._h, ctypes.c_void_p(0))
        return out, plvi.download(st.ptr, np.zeros(n * 2 * 16, np.int32)).reshape(n, 2, 16)
    return out


def test_mw_matches_oracle_and_sequential(plvi_lib, monkeypatch):
    frames = synth.batch(6, seed0=300)
    mw, st = _run(monkeypatch, frames, 256, stats=True)
    seq = _run(monkeypatch, frames, 0)
    for f in range(len(frames)):
        assert _same(mw[f], seq[f]), f"frame {f}: multi-wave != sequential kernel"
        exp = ol.line_extract(frames[f])
        assert _same(mw[f], exp), f"frame {f}: multi-wave != oracle"
    tot = st.sum(axis=(0, 1))
    # dispatched, dropped, regrown, exact, trivial, committed speculative
    assert tot[0] > 0 and tot[5] > 0 and tot[4] > 0, tot
    assert tot[5] + tot[2] <= tot[0]


def test_mw_real_and_extreme_frames(plvi_lib, monkeypatch):
    fr = real_frames()
    imgs = [fr["rgb1_gray"]] + [structured_frames()[k] for k in ("step", "checker", "stripes", "binary_noise")]
    frames = np.stack(imgs)
    mw = _run(monkeypatch, frames, 256)
    for f, img in enumerate(imgs):
        assert _same(mw[f], ol.line_extract(img)), f"image {f}"


def test_mw_euroc_752(plvi_lib, monkeypatch):
    fr = real_frames()
    frames = np.stack([fr["euroc1"], fr["euroc2"]])
    mw = _run(monkeypatch, frames, 256)
    for f in range(2):
        assert _same(mw[f], ol.line_extract(frames[f])), f"euroc{f + 1}"


def test_mw_flat_and_single_frame(plvi_lib, monkeypatch):
    flat = np.full((1, 480, 640), 77, np.uint8)
    assert len(_run(monkeypatch, flat, 256)[0][0]) == 0
    one = synth.batch(1, seed0=7)
    assert _same(_run(monkeypatch, one, 256)[0], ol.line_extract(one[0]))


@pytest.mark.parametrize("mw", [256, 0])
def test_rect_lanes_small_and_batch_grid(plvi_lib, monkeypatch, mw):
    """region2rect + get_theta (lsd.cpp:688-782) in lsd_rect_lanes_kernel
    (lane = region, with the nine multiply-adds lsd.cpp.o fuses) behind
    either region-growing kernel, at the small-batch grid (8 workgroups per
    (frame, octave)) and the batch grid: every frame equals the oracle."""
    st_ = structured_frames()
    frames = np.concatenate([synth.batch(17, seed0=900), np.stack([st_["checker"], st_["stripes"]])])
    for n in (2, len(frames)):
        got = _run(monkeypatch, frames[:n], mw)
        for f in range(n):
            kl, de, fn = ol.line_extract(frames[f])
            assert _same(got[f], (kl.astype(plvi.KEYLINE_DTYPE), de, fn)), f"n={n} frame {f}"


def test_mw_consecutive_launches(plvi_lib, monkeypatch):
    """One extractor, consecutive launches over different frames: the own-mark
    spill bitmaps are kept zero by every launch (never cleared in between),
    so no launch sees another frame's marks."""
    monkeypatch.setenv("PLVI_GROW_MW", "256")
    frames = synth.batch(4, seed0=520)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=2)
    lib = plvi.load()
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    for rep in range(2):
        for i in (0, 2, 1):  # frame pairs (0, 1), (2, 3), (1, 2)
            lx.extract_batch(buf.ptr + i * 640 * 480, 2, 640 * 480, 640)
            lib.plvi_device_synchronize()
            assert lx.errors() == 0
            out = _tables(lx, 2)
            for f in range(2):
                assert _same(out[f], ol.line_extract(frames[i + f])), f"rep {rep} pair {i} frame {f}"
    lx.close()


def test_mw_repeatable_against_sequential(plvi_lib, monkeypatch):
    """The multi-wave kernel's result must not depend on how its waves
    interleave: eight launches over the same 16 frames each equal the
    sequential kernel bit for bit (r06: an unlocked slot claim between a
    grower and the dispatcher once gave 2 differing frames in 480,
    tools/mw_stress.py, profiles/r06/mw_stress_*.txt)."""
    frames = synth.batch(16, seed0=5)
    seq = _run(monkeypatch, frames, 0)
    monkeypatch.setenv("PLVI_GROW_MW", "256")
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=16)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    for rep in range(8):
        lx.extract_batch(buf.ptr, 16, 640 * 480, 640)
        plvi_lib.plvi_device_synchronize()
        assert lx.errors() == 0
        out = _tables(lx, 16)
        bad = [f for f in range(16) if not _same(out[f], seq[f])]
        assert not bad, f"launch {rep}: frames {bad} differ from the sequential kernel"
    lx.close()
