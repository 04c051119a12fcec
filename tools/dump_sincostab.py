"""Dump glibc's __sincostab (sysdeps/ieee754/dbl-64/sincostab.c) from the host
libm into pl-vi-orbslam3_amd/csrc/glibc_sincostab.inc.

The table is 110 records of (sin(k/128) hi, lo, cos(k/128) hi, lo).  It is a
local symbol of libm.so.6, so it is located by its second record: the bytes of
the double sin(1/128) (Python's math.sin is this glibc's sin, and the record's
hi part is the double nearest sin(1/128)).  Run once on the build container;
the committed .inc is what the product compiles.  The values are checked
through plvi_sincos_glibc against glibc's sincos / sin / cos exhaustively over
region2rect's domain (tests/native/libm_check.cpp, mode r2rect).
"""
import math
import pathlib
import struct
import sys

LIBM = "/usr/lib/x86_64-linux-gnu/libm.so.6"
OUT = pathlib.Path(__file__).resolve().parent.parent / "pl-vi-orbslam3_amd" / "csrc" / "glibc_sincostab.inc"


def main():
    data = pathlib.Path(LIBM).read_bytes()
    key = struct.pack("<d", math.sin(1 / 128))
    hits = []
    i = data.find(key)
    while i != -1:
        hits.append(i)
        i = data.find(key, i + 1)
    # record 1 starts 32 bytes into the table; record 0 is (0, 0, 1, 0)
    base = None
    for h in hits:
        b = h - 32
        r0 = struct.unpack("<4d", data[b:b + 32])
        if r0 == (0.0, 0.0, 1.0, 0.0):
            base = b
    if base is None:
        sys.exit("table not found")
    vals = struct.unpack("<440d", data[base:base + 440 * 8])
    for k in range(110):
        assert vals[4 * k] == math.sin(k / 128) and vals[4 * k + 2] == math.cos(k / 128), k
    lines = [
        "// glibc 2.35 __sincostab (sysdeps/ieee754/dbl-64/sincostab.c): for k = 0..109",
        "// sin(k/128) hi, lo, cos(k/128) hi, lo.  Values dumped from this image's",
        "// libm.so.6 (tools/dump_sincostab.py), checked through plvi_sincos_glibc",
        "// against glibc's sincos / sin / cos (tests/native/libm_check.cpp).",
    ]
    for k in range(110):
        lines.append("    " + ", ".join(vals[4 * k + j].hex() for j in range(4)) + ",")
    OUT.write_text("\n".join(lines) + "\n")
    print(f"wrote {OUT} (table at file offset {base:#x})")


if __name__ == "__main__":
    main()
