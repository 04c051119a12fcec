"""bench.py's byte models and committed PMC traffic (CPU): the roofline
numerators are BASELINE.md §3's per-frame algorithmic bytes."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_blur_fast_bytes_is_baseline_blur_plus_fast_read_plus_copy():
    b = _bench()
    # 7x7 blur of 8 levels 1 901 064 (read + write),
    # FAST scoring read 950 532; the kernel also writes the score planes and
    # level 0's pyramid copy
    dims = b.level_dims(640, 480)
    planes = sum(w * h for w, h in dims)
    assert planes == 950_532
    assert b.blur_fast_bytes(640, 480) == 3_158_796 == planes + 2 * planes + 640 * 480


def test_end_to_end_bytes_match_baseline_totals():
    b = _bench()
    assert b.E2E_BYTES_640 == 15_972_194
    assert b.E2E_BYTES_752 == 18_775_975


def test_lsd_prep_bytes_counts_u8_in_and_f32_f64_out():
    b = _bench()
    # octave 0: 640x480 u8 -> 512x384 scaled; octave 1: 320x240 -> 256x192
    assert b.lsd_prep_bytes(640, 480) == 640 * 480 + 12 * 512 * 384 + 320 * 240 + 12 * 256 * 192


def test_committed_traffic_is_calibrated_and_near_algorithmic():
    b = _bench()
    t = b.committed_traffic(3072, "orb_blur_fast_kernel")
    assert t is not None
    alg = b.blur_fast_bytes(640, 480) * 3072
    assert 1.0 <= t / alg < 1.3  # measured 1.20
    assert b.committed_traffic(3071, "orb_blur_fast_kernel") is None
