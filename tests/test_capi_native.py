"""A C++ caller of the C-ABI (tests/native/capi_check.cpp) that includes only
include/plvi_frontend.h, the way the INTEGRATION.md shims do: it compiles
and links against the library on the CPU host (-std=c++11, the reference's
dialect), and on the GPU its ORB / line / LineMatcher::match outputs equal
the oracle's, with PLVI_E_EMPTY for empty images (ORBextractor.cc:1072)."""
import pathlib
import subprocess

import numpy as np
import pytest

import oracle_lib as ol
import plvi
from util import real_frames

ROOT = pathlib.Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "capi_check.cpp"
EXE = ROOT / "tests" / "native" / "_build" / "capi_check"


def build():
    if EXE.exists() and EXE.stat().st_mtime > max(SRC.stat().st_mtime, plvi.LIB_PATH.stat().st_mtime,
                                                    plvi.HEADER_PATH.stat().st_mtime):
        return EXE
    EXE.parent.mkdir(parents=True, exist_ok=True)
    libdir = plvi.LIB_PATH.parent
    subprocess.run(["g++", "-std=c++11", "-O1", "-Wall", "-Werror", f"-I{ROOT / 'include'}", str(SRC), "-o",
                    str(EXE), f"-L{libdir}", "-lplvi_frontend", f"-Wl,-rpath,{libdir}"], check=True)
    return EXE


def test_capi_check_compiles_and_links():
    exe = build()
    out = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True).stdout
    for name in ("plvi_orb_extract", "plvi_lines_extract", "plvi_line_match", "plvi_orb_errors"):
        assert name in out


@pytest.mark.gpu
def test_capi_check_matches_oracle(plvi_lib, tmp_path):
    exe = build()
    img = real_frames()["euroc1"]
    h, w = img.shape
    raw = tmp_path / "frame.raw"
    raw.write_bytes(np.ascontiguousarray(img).tobytes())
    out = tmp_path / "out.bin"
    subprocess.run([str(exe), str(raw), str(w), str(h), str(out)], check=True, timeout=120)
    buf = out.read_bytes()
    ns = int(np.frombuffer(buf, np.int32, 1)[0])
    st = np.frombuffer(buf, np.int32, ns, 4).tolist()
    (c_orb, e_null, e_zero, r_orb, r_oerr, oerr, n, mono, c_lx, r_lx, r_lerr, lerr, nl, nmatch,
     d_orb, d_lx) = st
    assert c_orb == 0 and c_lx == 0 and d_orb == 0 and d_lx == 0
    assert e_null == plvi.PLVI_E_EMPTY and e_zero == plvi.PLVI_E_EMPTY
    assert r_orb == 0 and r_oerr == 0 and oerr == 0 and r_lx == 0 and r_lerr == 0 and lerr == 0
    off = 4 + 4 * ns
    kps = np.frombuffer(buf, plvi.KEYPOINT_DTYPE, n, off)
    off += 28 * n
    desc = np.frombuffer(buf, np.uint8, 32 * n, off).reshape(n, 32)
    off += 32 * n
    kl = np.frombuffer(buf, plvi.KEYLINE_DTYPE, nl, off)
    off += 68 * nl
    ld = np.frombuffer(buf, np.uint8, 32 * nl, off).reshape(nl, 32)
    off += 32 * nl
    fn = np.frombuffer(buf, np.float64, 3 * nl, off).reshape(nl, 3)
    off += 24 * nl
    m12 = np.frombuffer(buf, np.int32, nl, off)
    me, ke, de = ol.orb_extract(img)
    assert mono == me and kps.tobytes() == ke.tobytes() and np.array_equal(desc, de)
    kle, lde, fne = ol.line_extract(img)
    assert kl.tobytes() == kle.tobytes() and np.array_equal(ld, lde) and fn.tobytes() == fne.tobytes()
    ne, mexp = ol.match(lde, lde[::-1].copy(), 0.9)
    assert nmatch == ne and np.array_equal(m12, mexp)
