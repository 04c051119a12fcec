"""Line front end parity: HIP path vs the CPU oracle, bit-exact.

KeyLine fields (all 17, bitwise), LBD descriptors byte-for-byte and the
normalised line equations (doubles, bitwise)."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import real_frames, structured_frames

pytestmark = pytest.mark.gpu


def _assert_same(got, exp, tag):
    kg, dg, fg = got
    ke, de, fe = exp
    assert len(kg) == len(ke), f"{tag}: n {len(kg)} != {len(ke)}"
    for f in ke.dtype.names:
        a, b = kg[f], ke[f]
        bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32)) if a.dtype.kind == "f" else np.flatnonzero(a != b)
        assert bad.size == 0, f"{tag}: field {f} differs at {bad[:10]} got {a[bad[:5]]} exp {b[bad[:5]]}"
    bad = np.flatnonzero((dg != de).any(axis=1))
    assert bad.size == 0, f"{tag}: descriptors differ at rows {bad[:10]}"
    bad = np.flatnonzero((fg.view(np.uint64) != fe.view(np.uint64)).any(axis=1))
    assert bad.size == 0, f"{tag}: line functions differ at rows {bad[:10]}"


@pytest.fixture(scope="module")
def lx640(plvi_lib):
    return plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=4)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lines_synthetic_640(lx640, seed):
    img = synth.frame(seed)
    _assert_same(lx640(img), ol.line_extract(img), f"synth{seed}")


def test_lines_real_euroc_752(plvi_lib):
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 752, 480)
    fr = real_frames()
    for k in ("euroc1", "euroc2"):
        _assert_same(lx(fr[k]), ol.line_extract(fr[k]), k)


def test_lines_real_rgb_640(lx640):
    img = real_frames()["rgb1_gray"]
    _assert_same(lx640(img), ol.line_extract(img), "rgb1_gray")


def test_lines_keep_all_and_100(plvi_lib):
    img = synth.frame(4)
    for nf in (0, 100):
        lx = plvi.Lineextractor(nf, 0, 0.8, 2, 2.0, 0, 640, 480)
        _assert_same(lx(img), ol.line_extract(img, nfeatures=nf), f"nfeatures={nf}")


def test_lines_flat_image(lx640):
    flat = np.full((480, 640), 77, np.uint8)
    kg, dg, fg = lx640(flat)
    ke, de, fe = ol.line_extract(flat)
    assert len(kg) == len(ke) == 0


def test_lines_pyramid_level1(lx640):
    img = synth.frame(8)
    lx640(img)
    s = img.astype(np.int32)
    tot = s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2]
    assert np.array_equal(lx640.pyramid_level(1), ((tot + 2) >> 2).astype(np.uint8))


def test_lines_batch_equals_single(lx640):
    frames = synth.batch(4, seed0=40)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    lx640.extract_batch(buf.ptr, 4, 640 * 480, 640)
    plvi.load().plvi_device_synchronize()
    klp, dep, fnp, cop, cap = lx640.outputs()
    cnt = plvi.download(cop, np.zeros(4, np.int32))
    kl = plvi.download(klp, np.zeros(4 * cap, plvi.KEYLINE_DTYPE))
    de = plvi.download(dep, np.zeros((4 * cap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((4 * cap, 3), np.float64))
    for f in range(4):
        s = slice(f * cap, f * cap + cnt[f])
        _assert_same((kl[s], de[s], fn[s]), ol.line_extract(frames[f]), f"batch{f}")


@pytest.mark.parametrize("lds,rb,rd", [(6144, "64", None), (6144, "2", None), (6144, "8", "0"),
                                       (12288, "64", "2"), (40960, "16", None), (40960, "1024", None)])
def test_lines_grow_window_budgets(plvi_lib, monkeypatch, lds, rb, rd):
    """PLVI_GROW_LDS / _RB / _RD pick the region-growing LDS windows (USED
    bits ring of RB rows, angle ring of R rows or none, the 1024-entry queue
    at the larger budgets): every choice gives the oracle's lines, at 640 px
    (odd batch) and at the 752 px EuRoC width (BASELINE C4)."""
    monkeypatch.setenv("PLVI_GROW_MW", "0")  # the sequential (large-batch) kernel
    monkeypatch.setenv("PLVI_GROW_LDS", str(lds))
    monkeypatch.setenv("PLVI_GROW_RB", rb)
    if rd is not None:
        monkeypatch.setenv("PLVI_GROW_RD", rd)
    else:
        monkeypatch.delenv("PLVI_GROW_RD", raising=False)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=3)
    frames = synth.batch(3, seed0=60)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    lx.extract_batch(buf.ptr, 3, 640 * 480, 640)
    plvi.load().plvi_device_synchronize()
    klp, dep, fnp, cop, cap = lx.outputs()
    cnt = plvi.download(cop, np.zeros(3, np.int32))
    kl = plvi.download(klp, np.zeros(3 * cap, plvi.KEYLINE_DTYPE))
    de = plvi.download(dep, np.zeros((3 * cap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((3 * cap, 3), np.float64))
    for f in range(3):
        s = slice(f * cap, f * cap + cnt[f])
        _assert_same((kl[s], de[s], fn[s]), ol.line_extract(frames[f]), f"lds{lds} batch{f}")
    assert lx.errors() == 0
    lx752 = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 752, 480)
    img = real_frames()["euroc1"]
    _assert_same(lx752(img), ol.line_extract(img), f"lds{lds} euroc1")


@pytest.mark.parametrize("name", ["step", "checker", "stripes", "binary_noise"])
def test_lines_structured_extremes(lx640, name):
    img = structured_frames()[name]
    _assert_same(lx640(img), ol.line_extract(img), name)


@pytest.mark.parametrize("tpw", ["2", "0"])
def test_lines_grow_tasks_per_wave(plvi_lib, monkeypatch, tpw):
    """PLVI_GROW_TPW=2 runs two growth tasks per wave of the large-batch kernel
    (octave 0 then octave 1 of a frame, the LOOP form); 0 selects the r06
    in-schedule rule.  Either gives the oracle's lines (odd batch: the last
    wave holds one task)."""
    monkeypatch.setenv("PLVI_GROW_MW", "0")
    monkeypatch.setenv("PLVI_GROW_TPW", tpw)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=3)
    frames = synth.batch(3, seed0=80)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    lx.extract_batch(buf.ptr, 3, 640 * 480, 640)
    plvi.load().plvi_device_synchronize()
    klp, dep, fnp, cop, cap = lx.outputs()
    cnt = plvi.download(cop, np.zeros(3, np.int32))
    kl = plvi.download(klp, np.zeros(3 * cap, plvi.KEYLINE_DTYPE))
    de = plvi.download(dep, np.zeros((3 * cap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((3 * cap, 3), np.float64))
    for f in range(3):
        s = slice(f * cap, f * cap + cnt[f])
        _assert_same((kl[s], de[s], fn[s]), ol.line_extract(frames[f]), f"tpw {tpw} frame {f}")
    assert lx.errors() == 0
