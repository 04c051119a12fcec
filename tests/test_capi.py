"""C-ABI library: loads on a CPU-only host and exports every declared symbol."""
import ctypes
import subprocess

import plvi


def test_library_exports_every_header_symbol():
    lib = plvi.load()
    names = plvi.exported_symbols()
    assert "plvi_orb_extract" in names and "plvi_hamming_knn2_batch" in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", str(plvi.LIB_PATH)], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}" in out, n


def test_library_contains_gfx950_code_only():
    out = subprocess.run(["strings", str(plvi.LIB_PATH)], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_version_and_no_device_does_not_crash():
    lib = plvi.load()
    assert b"gfx950" in lib.plvi_version()
    assert lib.plvi_device_count() >= 0


def test_keypoint_and_keyline_layouts():
    assert plvi.KEYPOINT_DTYPE.itemsize == 28  # cv::KeyPoint
    assert plvi.KEYLINE_DTYPE.itemsize == 68   # line_descriptor::KeyLine
