"""The oracle's GridStructure / LineIterator restatements against the
reference's own code (SURVEY §8c pin).

/root/reference/src/gridStructure.cpp and src/LineIterator.cpp include only
the standard library, so oracle/ref/Makefile compiles them in place,
unmodified, into oracle/_ref/libref_grid.so (with oracle/ref/grid_driver.cpp:
C entry points only).  Compared here:

* getLineCoords / LineIterator (gridStructure.cpp:32-40, LineIterator.cpp:31-73)
  with the oracle's `line_coords` (oracle/stereo_oracle.cpp), which the stereo
  line grid (f4) and the HIP `line_iterate` are checked against;
* GridStructure::get at the start and end cells into one unordered_set, as
  LineMatcher::matchGrid does (LineMatcher.cpp:226-227), with the oracle's
  `grid_get` (oracle/match_oracle.cpp, feeding a23 / f4 / f6) in its
  range_hint = 0 mode -- the rule of this host's libstdc++, which the _ref
  build uses.  The reference's own GCC 9 rule (range_hint = 1, the product
  default) is pinned by tests/test_ref_objects.py::
  test_grid_get_passes_the_range_length_as_rehash_hint and
  tests/native/uset_check.cpp.

Skips where /root/reference is absent (the GPU box).
"""
import ctypes
import os
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_lib
import util

ROOT = pathlib.Path(__file__).resolve().parent.parent
REF_SRC = pathlib.Path("/root/reference/src")
LIB = ROOT / "oracle" / "_ref" / "libref_grid.so"

pytestmark = pytest.mark.skipif(not (REF_SRC / "gridStructure.cpp").exists() or os.environ.get("PLVI_SKIP_REF") == "1",
                                reason="/root/reference absent (or PLVI_SKIP_REF=1)")


@pytest.fixture(scope="module")
def ref():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle" / "ref")], check=True)
    lib = ctypes.CDLL(str(LIB))
    V, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.ref_line_coords.argtypes = [D, D, D, D, V, I]
    lib.ref_line_coords.restype = I
    lib.ref_grid_candidates.argtypes = [I, I, V, V, I, I, I, I, I, I, I, I, V, I]
    lib.ref_grid_candidates.restype = I
    lib.ref_grid_at_in_bounds.argtypes = [I, I, I, I]
    lib.ref_grid_at_in_bounds.restype = I
    return lib


def _segments(seed, n=3000):
    """Grid-coordinate segments as Frame::ComputeStereoMatches_Lines feeds them
    (keyline endpoints x 64/W, 48/H), plus degenerate and boundary ones."""
    rng = np.random.default_rng(seed)
    segs = [tuple(v) for v in np.stack([rng.uniform(-3, 68, n), rng.uniform(-3, 52, n),
                                        rng.uniform(-3, 68, n), rng.uniform(-3, 52, n)], 1)]
    segs += [(5.0, 5.0, 5.0, 5.0), (0.0, 0.0, 63.99, 0.0), (3.5, 0.0, 3.5, 47.5), (10.5, 10.5, 20.5, 20.5),
             (20.5, 20.5, 10.5, 10.5), (0.49, 7.5, 40.5, 8.49), (-0.5, -0.5, 2.5, 1.5), (63.0, 47.0, 0.0, 0.0),
             (1.0, 2.0, 1.0 + 1e-12, 30.0), (30.0, 1.0, 2.0, 1.0 + 1e-13)]
    # integer and half-integer endpoints (the truncation / error-sign edges)
    k = rng.integers(0, 128, (400, 4)) / 2.0
    segs += [tuple(v) for v in k]
    return segs


def test_line_coords_equal_reference(ref):
    for seed in (0, 1):
        for s in _segments(seed):
            got = oracle_lib.line_coords(*s)
            want = oracle_lib.line_coords(*s, lib=ref, fn="ref_line_coords")
            assert got == want, s
            assert util.line_iterator(*s) == want, s  # the Python restatement tests use


def test_line_coords_on_real_keylines(ref):
    frames = util.real_frames()
    for name in sorted(frames)[:4]:
        kl, _, _ = oracle_lib.line_extract(frames[name])
        iw, ih = 64 / 640, 48 / 480
        for k in kl:
            s = (float(k["startPointX"]) * iw, float(k["startPointY"]) * ih, float(k["endPointX"]) * iw,
                 float(k["endPointY"]) * ih)
            assert oracle_lib.line_coords(*s) == oracle_lib.line_coords(*s, lib=ref, fn="ref_line_coords")


def _random_grid(rng, cols=64, rows=48, n=300, dup=True):
    grid = [[[] for _ in range(rows)] for _ in range(cols)]
    for i in range(n):
        x0, y0 = rng.uniform(0, cols), rng.uniform(0, rows)
        x1, y1 = np.clip(x0 + rng.normal(0, 12), 0, cols - 0.01), np.clip(y0 + rng.normal(0, 9), 0, rows - 0.01)
        for (x, y) in util.line_iterator(x0, y0, x1, y1):
            if 0 <= x < cols and 0 <= y < rows:
                grid[x][y].append(i)
    if dup:  # the same index in many cells, and repeated within a cell
        for _ in range(200):
            x, y = rng.integers(0, cols), rng.integers(0, rows)
            grid[x][y].extend(rng.integers(0, n, rng.integers(1, 5)).tolist())
    return grid


@pytest.mark.parametrize("seed", range(4))
def test_grid_candidates_equal_reference(ref, seed):
    rng = np.random.default_rng(100 + seed)
    grid = _random_grid(rng)
    windows = [((7, 0), (2, 2)), ((2, 2), (2, 2)), ((0, 0), (0, 0)), ((10, 10), (10, 10))]
    for _ in range(250):
        sp = (int(rng.integers(-3, 67)), int(rng.integers(-3, 51)))
        ep = (int(rng.integers(-3, 67)), int(rng.integers(-3, 51)))
        w = windows[int(rng.integers(0, len(windows)))]
        got = oracle_lib.grid_candidates(grid, sp, ep, w, range_hint=0)
        want = oracle_lib.grid_candidates(grid, sp, ep, w, lib=ref, fn="ref_grid_candidates")
        assert got == want, (sp, ep, w)


def test_grid_candidates_on_stereo_case(ref):
    lines1, _, grid, _, _ = util.stereo_line_case(5)
    for l in lines1:
        sp, ep = (int(l[0]), int(l[1])), (int(l[2]), int(l[3]))
        assert oracle_lib.grid_candidates(grid, sp, ep, range_hint=0) == \
            oracle_lib.grid_candidates(grid, sp, ep, lib=ref, fn="ref_grid_candidates")


def test_grid_at_bounds(ref):
    """at(x, y) outside the grid is the shared out_of_bounds list: the stereo
    grid build drops such LineIterator pixels (the kernels' bounds test)."""
    for (x, y, inb) in [(0, 0, 1), (63, 47, 1), (64, 0, 0), (0, 48, 0), (-1, 5, 0), (5, -1, 0)]:
        assert ref.ref_grid_at_in_bounds(64, 48, x, y) == inb
