"""The product's glibc-faithful math (csrc/plvi_math.h) vs the host glibc,
exhaustively where the domain is finite."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "libm_check.cpp"
BIN = ROOT / "tests" / "native" / "_build" / "libm_check"


@pytest.fixture(scope="module")
def libm_check():
    BIN.parent.mkdir(exist_ok=True)
    hdr = ROOT / "pl-vi-orbslam3_amd" / "csrc" / "plvi_math.h"
    if not BIN.exists() or BIN.stat().st_mtime < max(SRC.stat().st_mtime, hdr.stat().st_mtime):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-pthread", "-o",
                        str(BIN), str(SRC), str(ROOT / "oracle" / "cvprim.cpp"), "-lm"], check=True)
    return str(BIN)


def _run(binp, *args):
    r = subprocess.run([binp, *args], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout
    return r.stdout


def test_sinf_cosf_every_float(libm_check):
    out = _run(libm_check, "sincosf")          # all 2^32 bit patterns, both functions
    assert "checked=4294967296" in out


def test_lsd_double_cos_sin_every_float_angle(libm_check):
    _run(libm_check, "lsdangles")              # float(cos/sin(deg*pi/180)) for every float deg in [0,360]


def test_region2rect_sincos_double_bitwise(libm_check):
    # region2rect's sincos(theta) (lsd.cpp:710-711) as DOUBLES, theta = T*pi/180
    # for every float T in [0, 360] and theta + pi: 2 271 739 906 arguments
    out = _run(libm_check, "r2rect")
    assert "checked=2271739906" in out


def test_glibc_sincos_sampled_doubles(libm_check):
    _run(libm_check, "sincosd", "30000000")    # |x| < 105414350, all binades


def test_atan2f_sampled(libm_check):
    _run(libm_check, "atan2f", "30000000")


def test_branch_free_sincosf_every_float(libm_check):
    _run(libm_check, "sincospos")              # plvi_sincosf_pos vs glibc sinf/cosf, every float in [0, 120)


def test_fast_atan2_select_form(libm_check):
    _run(libm_check, "fastatan2", "30000000")  # branch-free device cv::fastAtan2 vs the oracle restatement


# ---------------------------------------------------------------- on device
DSRC = ROOT / "tests" / "native" / "libm_device_check.hip"
DBIN = ROOT / "tests" / "native" / "_build" / "libm_device_check"


def build_device_check():
    """hipcc with the library's flags (gfx950, -O3, -ffp-contract=off), linked
    to the oracle for cv::fastAtan2."""
    hdr = ROOT / "pl-vi-orbslam3_amd" / "csrc" / "plvi_math.h"
    olib = ROOT / "oracle" / "_build"
    if not (olib / "liboracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    if not DBIN.exists() or DBIN.stat().st_mtime < max(DSRC.stat().st_mtime, hdr.stat().st_mtime):
        DBIN.parent.mkdir(exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-fast-math", "-pthread", "-o", str(DBIN), str(DSRC), f"-L{olib}", "-loracle",
                        f"-Wl,-rpath,{olib}"], check=True)
    return str(DBIN)


def test_device_libm_check_builds():
    assert pathlib.Path(build_device_check()).exists()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,args,count", [
    ("sincosf", (), 4294967296),          # every float bit pattern, sinf and cosf
    ("sincospos", (), None),              # branch-free sincosf, every float in [0, 120)
    ("lsdangles", (), None),              # float(cos/sin(+-deg*pi/180)), every float deg in [0, 360]
    ("r2rect", (), None),                 # region2rect's double sincos(theta), theta + pi: every float deg
    ("atan2f", ("30000000",), 30000000),
    ("fastatan2", ("30000000",), 30000000),
])
def test_device_libm_matches_host_glibc(mode, args, count):
    out = _run(build_device_check(), mode, *args)
    if count:
        assert f"checked={count}" in out
