"""ORB parity: HIP path (through the C-ABI) vs the CPU oracle, bit-exact.

Keypoints compare every cv::KeyPoint field bitwise (x, y, size, angle,
response, octave, class_id) in the reference's slot order; descriptors
byte-for-byte; monoIndex exactly."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import real_frames, structured_frames

pytestmark = pytest.mark.gpu


def _assert_same(got, exp, tag):
    mg, kg, dg = got
    me, ke, de = exp
    assert mg == me, f"{tag}: monoIndex {mg} != {me}"
    assert len(kg) == len(ke), f"{tag}: n {len(kg)} != {len(ke)}"
    for f in ke.dtype.names:
        a, b = kg[f], ke[f]
        bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32)) if a.dtype.kind == "f" else np.flatnonzero(a != b)
        assert bad.size == 0, f"{tag}: field {f} differs at {bad[:10]} got {a[bad[:5]]} exp {b[bad[:5]]}"
    bad = np.flatnonzero((dg != de).any(axis=1))
    assert bad.size == 0, f"{tag}: descriptors differ at rows {bad[:10]}"


@pytest.fixture(scope="module")
def orb640(plvi_lib):
    return plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=8)


@pytest.fixture(scope="module")
def orb752(plvi_lib):
    return plvi.ORBextractor(1000, 1.2, 8, 20, 7, 752, 480, max_batch=2)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_orb_synthetic_640(orb640, seed):
    img = synth.frame(seed)
    _assert_same(orb640(img, None, (0, 0)), ol.orb_extract(img), f"synth{seed}")


def test_orb_pyramid_matches_oracle(orb640):
    img = synth.frame(5)
    orb640(img, None, (0, 0))
    for level in range(8):
        exp = ol.orb_stage(img, level)
        got = orb640.pyramid_level(level)
        assert np.array_equal(got, exp["pyr"]), f"level {level}"


@pytest.mark.parametrize("pad", [5, 0])
@pytest.mark.parametrize("mode", ["0", "100000"])
@pytest.mark.parametrize("wh", [(640, 480), (752, 480), (641, 479)])
def test_orb_pyramid_builders_batch(plvi_lib, monkeypatch, mode, wh, pad):
    """Both pyramid builders -- the streaming kernel (PLVI_PYR_LEVELWISE=0: every batch) and the
    level-by-level launches (PLVI_PYR_LEVELWISE=100000) -- give the oracle's levels for every frame of a
    batch read from a row-padded (pad 5: level 0 copied into the pyramid) or packed (pad 0: level 0 is a
    view of the caller's frames) device buffer, and the oracle's keypoints and descriptors."""
    monkeypatch.setenv("PLVI_PYR_LEVELWISE", mode)
    w, h = wh
    imgs = [synth.frame(40 + k, w, h) for k in range(3)]
    imgs.append(structured_frames(w, h)["checker"])
    B, stride = len(imgs), w + pad  # padded rows: frames as a strided view
    frames = np.zeros((B, h, stride), np.uint8)
    for k, im in enumerate(imgs):
        frames[k, :, :w] = im
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    ext = plvi.ORBextractor(1000, 1.2, 8, 20, 7, w, h, max_batch=B)
    ext.extract_batch(buf.ptr, B, h * stride, stride)
    plvi_lib.plvi_device_synchronize()
    assert ext.errors() == 0
    p0, fs0, w0, h0 = ext.pyramid_device(0)
    assert (w0, h0) == (w, h)
    if pad == 0:
        assert (p0, fs0) == (buf.ptr, h * stride), "packed frames: level 0 is a view of the batch"
    else:
        assert p0 != buf.ptr and fs0 == w * h
    for k, im in enumerate(imgs):
        for level in range(8):
            exp = ol.orb_stage(im, level)
            assert np.array_equal(ext.pyramid_level(level, k), exp["pyr"]), f"mode {mode} frame {k} level {level}"
    kp_p, de_p, co_p, mo_p, cap = ext.outputs()
    cnt = plvi.download(co_p, np.zeros(B, np.int32))
    mono = plvi.download(mo_p, np.zeros(B, np.int32))
    kps = plvi.download(kp_p, np.zeros(B * cap, plvi.KEYPOINT_DTYPE))
    desc = plvi.download(de_p, np.zeros((B * cap, 32), np.uint8))
    for k, im in enumerate(imgs):
        s = slice(k * cap, k * cap + cnt[k])
        _assert_same((int(mono[k]), kps[s], desc[s]), ol.orb_extract(im), f"mode {mode} frame {k}")
    ext.close()


def test_orb_level0_copy_switch(plvi_lib, monkeypatch):
    """PLVI_ORB_L0_COPY=1 keeps the r05 layout (level 0 copied into the pyramid buffer) for packed
    frames too; both layouts give the oracle's outputs."""
    frames = synth.batch(3, seed0=60)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    for copy in ("0", "1"):
        monkeypatch.setenv("PLVI_ORB_L0_COPY", copy)
        ext = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=3)
        ext.extract_batch(buf.ptr, 3, 640 * 480, 640)
        plvi_lib.plvi_device_synchronize()
        p0 = ext.pyramid_device(0)[0]
        assert (p0 == buf.ptr) == (copy == "0")
        for k in range(3):
            assert np.array_equal(ext.pyramid_level(0, k), frames[k])
        kp_p, de_p, co_p, mo_p, cap = ext.outputs()
        cnt = plvi.download(co_p, np.zeros(3, np.int32))
        mono = plvi.download(mo_p, np.zeros(3, np.int32))
        kps = plvi.download(kp_p, np.zeros(3 * cap, plvi.KEYPOINT_DTYPE))
        desc = plvi.download(de_p, np.zeros((3 * cap, 32), np.uint8))
        for k in range(3):
            s = slice(k * cap, k * cap + cnt[k])
            _assert_same((int(mono[k]), kps[s], desc[s]), ol.orb_extract(frames[k]), f"copy {copy} frame {k}")
        ext.close()


def test_orb_octree_memory_scan_path(plvi_lib, monkeypatch):
    """PLVI_ORB_OCT_LDS=0 sends every level's octree down the path used when a
    level's candidate list exceeds the LDS stage (counts and node maxima by
    scanning the list in memory instead of partitioned per-node ranges); both
    paths give the oracle's outputs, on smooth frames and on binary noise."""
    frames = np.concatenate([synth.batch(2, seed0=70),
                             np.random.default_rng(9).integers(0, 256, size=(1, 480, 640), dtype=np.uint8)])
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    for lds in ("0", "1536"):
        monkeypatch.setenv("PLVI_ORB_OCT_LDS", lds)
        ext = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=3)
        ext.extract_batch(buf.ptr, 3, 640 * 480, 640)
        plvi_lib.plvi_device_synchronize()
        kp_p, de_p, co_p, mo_p, cap = ext.outputs()
        cnt = plvi.download(co_p, np.zeros(3, np.int32))
        mono = plvi.download(mo_p, np.zeros(3, np.int32))
        kps = plvi.download(kp_p, np.zeros(3 * cap, plvi.KEYPOINT_DTYPE))
        desc = plvi.download(de_p, np.zeros((3 * cap, 32), np.uint8))
        for k in range(3):
            s = slice(k * cap, k * cap + cnt[k])
            _assert_same((int(mono[k]), kps[s], desc[s]), ol.orb_extract(frames[k]), f"oct lds {lds} frame {k}")
        ext.close()


def test_orb_real_euroc_752(orb752):
    fr = real_frames()
    for k in ("euroc1", "euroc2"):
        _assert_same(orb752(fr[k]), ol.orb_extract(fr[k]), k)


def test_orb_real_rgb_640(orb640):
    img = real_frames()["rgb1_gray"]
    _assert_same(orb640(img), ol.orb_extract(img), "rgb1_gray")


def test_orb_lapping_area_slots(orb640):
    img = synth.frame(6)
    for lap in [(0, 1000), (100, 300), (0, 0)]:
        _assert_same(orb640(img, None, lap), ol.orb_extract(img, lap=lap), f"lap{lap}")


def test_orb_ini_extractor_5000(plvi_lib):
    ext = plvi.ORBextractor(5000, 1.2, 8, 20, 7, 640, 480)
    img = synth.frame(7)
    _assert_same(ext(img), ol.orb_extract(img, nfeatures=5000), "ini5000")


def test_orb_flat_and_noise_edge_cases(orb640):
    flat = np.full((480, 640), 128, np.uint8)
    _assert_same(orb640(flat), ol.orb_extract(flat), "flat")
    rng = np.random.default_rng(0)
    noise = rng.integers(0, 256, size=(480, 640), dtype=np.uint8)
    _assert_same(orb640(noise), ol.orb_extract(noise), "noise")


def test_orb_empty_image_returns_minus_one(orb640):
    mono, k, d = orb640(np.zeros((0, 0), np.uint8))
    assert mono == -1 and len(k) == 0


def test_orb_batch_equals_single(orb640):
    frames = synth.batch(8, seed0=20)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    orb640.extract_batch(buf.ptr, 8, 640 * 480, 640)
    plvi.load().plvi_device_synchronize()
    kp_p, de_p, co_p, mo_p, cap = orb640.outputs()
    cnt = plvi.download(co_p, np.zeros(8, np.int32))
    mono = plvi.download(mo_p, np.zeros(8, np.int32))
    kps = plvi.download(kp_p, np.zeros(8 * cap, plvi.KEYPOINT_DTYPE))
    desc = plvi.download(de_p, np.zeros((8 * cap, 32), np.uint8))
    for f in range(8):
        exp = ol.orb_extract(frames[f])
        got = (int(mono[f]), kps[f * cap:f * cap + cnt[f]], desc[f * cap:f * cap + cnt[f]])
        _assert_same(got, exp, f"batch{f}")


@pytest.mark.parametrize("name", ["step", "checker", "stripes", "binary_noise"])
def test_orb_structured_extremes(orb640, name):
    img = structured_frames()[name]
    _assert_same(orb640(img), ol.orb_extract(img), name)


def _batch_tables(orb, batch):
    n = len(batch)
    buf = plvi.DeviceBuffer(batch.nbytes)
    buf.upload(np.ascontiguousarray(batch))
    orb.extract_batch(buf.ptr, n, 640 * 480, 640)
    plvi.load().plvi_device_synchronize()
    kp_p, de_p, co_p, mo_p, cap = orb.outputs()
    cnt = plvi.download(co_p, np.zeros(n, np.int32))
    mono = plvi.download(mo_p, np.zeros(n, np.int32))
    kps = plvi.download(kp_p, np.zeros(n * cap, plvi.KEYPOINT_DTYPE))
    desc = plvi.download(de_p, np.zeros((n * cap, 32), np.uint8))
    return [(int(mono[f]), kps[f * cap:f * cap + cnt[f]], desc[f * cap:f * cap + cnt[f]]) for f in range(n)]


def test_orb_octree_overflow_then_normal_batch(plvi_lib):
    """An octree overflow (forced with the plvi_orb_debug_node_cap hook) flags
    its frames and writes no level keypoints; the next normal batch through
    the same handle (its candidate lists restart from zero) is the oracle's
    bit for bit."""
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=4)
    lib = plvi.load()
    noise = np.random.default_rng(5).integers(0, 256, size=(4, 480, 640), dtype=np.uint8)
    frames = synth.batch(4, seed0=60)
    assert lib.plvi_orb_debug_node_cap(orb._h, 6) == 0
    _batch_tables(orb, noise)
    flags = orb.errors(per_frame=True)
    assert all(int(v) & 1 for v in np.atleast_1d(flags)[:4]), flags
    assert lib.plvi_orb_debug_node_cap(orb._h, 0) == 0
    for f, got in enumerate(_batch_tables(orb, frames)):
        _assert_same(got, ol.orb_extract(frames[f]), f"after overflow f={f}")
    assert orb.errors() == 0
    orb.close()


def test_orb_candidate_lists_reuse_across_batches(orb640):
    """The NMS candidate lists (appended in arbitrary cell order, counted and
    maximised per octree node, lists of the dense levels beyond the octree
    wave's LDS read from memory) are reused across batches: a batch after a
    larger, candidate-dense one (binary noise) and a shorter batch after it
    must still match the oracle frame by frame."""
    noise = np.random.default_rng(3).integers(0, 256, size=(8, 480, 640), dtype=np.uint8)
    frames = synth.batch(8, seed0=40)
    for batch in (noise, frames[:3], frames[3:8], noise[:1], frames[:8]):
        n = len(batch)
        buf = plvi.DeviceBuffer(batch.nbytes)
        buf.upload(np.ascontiguousarray(batch))
        orb640.extract_batch(buf.ptr, n, 640 * 480, 640)
        plvi.load().plvi_device_synchronize()
        kp_p, de_p, co_p, mo_p, cap = orb640.outputs()
        cnt = plvi.download(co_p, np.zeros(n, np.int32))
        mono = plvi.download(mo_p, np.zeros(n, np.int32))
        kps = plvi.download(kp_p, np.zeros(n * cap, plvi.KEYPOINT_DTYPE))
        desc = plvi.download(de_p, np.zeros((n * cap, 32), np.uint8))
        for f in range(n):
            got = (int(mono[f]), kps[f * cap:f * cap + cnt[f]], desc[f * cap:f * cap + cnt[f]])
            _assert_same(got, ol.orb_extract(batch[f]), f"reuse n={n} f={f}")
