"""LineMatcher::matchGrid (src/LineMatcher.cpp:191-272) + GridStructure::get.

The oracle uses the host's real std::unordered_set for both candidate
orders: range_hint=0 (GCC >= 11 insert(first, last), this host) and
range_hint=1 (the reference's GCC 9 rule: the range length as rehash hint),
which it runs through libstdc++ 11's merge() -- the same hint loop inside the
host library (oracle/match_oracle.cpp) -- so both orders are checked against
real container code, independently of the product's emulation
(csrc/stl_uset.h).  The order decides best/second among equal distances."""
import subprocess
import pathlib

import numpy as np
import pytest

import oracle_lib
import util

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_unordered_set_emulation_matches_host_libstdcxx():
    src = ROOT / "tests" / "native" / "uset_check.cpp"
    exe = ROOT / "tests" / "native" / "_build" / "uset_check"
    exe.parent.mkdir(exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(src)], check=True)
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches=0" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([str(exe), "20000", "gcc10"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches=0" in r.stdout, r.stdout + r.stderr


def test_gcc10_range_insert_changes_order():
    """The hint matters: one 12-line cell inserted into an empty set gets 13
    buckets at once under GCC <= 10 (hint 12) but grows 1 -> 13 -> ... element
    by element under GCC 11, and the two iteration orders differ."""
    cells = [[40, 3, 27, 14, 1, 52, 9, 33, 18, 6, 45, 22], [7, 60, 2]]
    a, b = oracle_lib.uset_order(cells, 0), oracle_lib.uset_order(cells, 1)
    assert sorted(a) == sorted(b) and a != b


def test_oracle_gcc10_order_equals_emulation_on_cases():
    """oracle (real container via merge) vs the product emulation compiled
    on the host, on the candidate sets of the tie-heavy stereo cases."""
    for seed in range(3):
        lines1, _, grid, _, _ = util.stereo_line_case(seed, n=150)
        cells = [grid[x][y] for x in range(20, 44) for y in range(10, 30)]
        assert len(oracle_lib.uset_order(cells, 1)) == len({i for c in cells for i in c})


def test_oracle_match_grid_basic():
    lines1, desc1, grid, desc2, dirs = util.stereo_line_case(0, n=120)
    n, m = oracle_lib.match_grid(lines1, desc1, grid, desc2, dirs)
    assert n == int((m >= 0).sum()) and n > 30
    # mutual consistency: no right line is used twice
    used = m[m >= 0]
    assert len(used) == len(set(used.tolist()))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_match_grid_matches_oracle(seed):
    import plvi
    case = util.stereo_line_case(seed, n=150 + 40 * seed, ties=seed % 2 == 0)
    n_ref, m_ref = oracle_lib.match_grid(*case)
    n, m = plvi.LineMatcher.matchGrid(*case, range_hint=0)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_match_grid_gcc10_order_matches_oracle(seed):
    """range_hint=1 (the shipped default: GCC 9's range-insert order) on
    tie-heavy grids (duplicated right lines and descriptors)."""
    import plvi
    case = util.stereo_line_case(100 + seed, n=150 + 40 * seed, ties=True)
    n_ref, m_ref = oracle_lib.match_grid(*case, range_hint=1)
    n, m = plvi.LineMatcher.matchGrid(*case, range_hint=1)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


@pytest.mark.gpu
def test_match_grid_degenerate_lines_and_empty():
    import plvi
    lines1, desc1, grid, desc2, dirs = util.stereo_line_case(11, n=80)
    lines1[:10, 2:] = lines1[:10, :2]  # zero-length lines: NaN direction keeps every candidate
    n_ref, m_ref = oracle_lib.match_grid(lines1, desc1, grid, desc2, dirs)
    n, m = plvi.LineMatcher.matchGrid(lines1, desc1, grid, desc2, dirs, range_hint=0)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)
    empty = [[[] for _ in range(48)] for _ in range(64)]
    n, m = plvi.LineMatcher.matchGrid(lines1, desc1, empty, desc2, dirs, range_hint=1)
    assert n == 0 and (m == -1).all()


# ------------------------------------ LineMatcher::SearchByProjection (LineMatcher.cpp:274-372)
def test_oracle_line_search_projection_sanity():
    case = util.line_proj_case(0)
    for hint in (0, 1):
        n, m = oracle_lib.line_search_projection(case, 3.0, float(np.float32(np.pi / 8)), hint)
        assert n >= (m >= 0).sum() > 20
        assert (m[case["cur_blocked"] == 1] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,hint", [(0, 3.0, 1), (1, 5.0, 1), (2, 3.0, 0), (3, 5.0, 0), (4, 8.0, 1)])
def test_line_search_projection_matches_oracle(seed, th, hint):
    import plvi
    case = util.line_proj_case(seed)
    angth = float(np.float32(np.pi / 8))
    ne, me = oracle_lib.line_search_projection(case, th, angth, hint)
    ng, mg = plvi.LineMatcher.SearchByProjection(util.line_proj_params(case, th, angth, hint), case["cur_angle"],
                                                 case["cur_desc"], case["grid"], case["last_flags"], case["x3dc"],
                                                 case["last_octave"], case["ml_desc"], case["cur_blocked"])
    assert ng == ne
    np.testing.assert_array_equal(mg, me)
