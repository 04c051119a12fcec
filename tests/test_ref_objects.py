"""Static pins from the reference's own compiled objects.

The reference ships its build tree: the objects of its own library
(build/CMakeFiles/ORB_SLAM3-Relocalization.dir/src/*.o, GCC 9.4, `-O3
-std=c++11 -march=native`) and of the vendored line_descriptor library
(Thirdparty/line_descriptor/build/.../linedesc.dir/src/*.o, `-O3
-mtune=native`).  They are never run or loaded: these tests only read them
with objdump / readelf, and pin the arithmetic facts the oracle (and the HIP
kernels) restate:

* the compiler: GCC 9.4, i.e. libstdc++ 9, whose unordered_set range insert
  passes the remaining range length as the rehash hint (the `range_hint=1`
  default of matchGrid), visible in GridStructure::get itself;
* which multiply-adds the build fused.  GCC's C++ front end contracts
  `a*b + c` into one FMA even under -std=c++11, so with -march=native the
  reference's own code is NOT one IEEE op per operator: every fused site on
  the path is listed below by function, with the instruction window that
  shows which product is fused (oracle/ref_fma.h, csrc/plvi_math.h rfma);
  every other path function holds no fused operation;
* the line_descriptor objects (LBD, KeyLine assembly) hold no fused
  operation and no VEX instruction at all (plain SSE2), and call the float
  libm functions the oracle assumes (cosf, sinf, roundf, sqrtf, atan2f);
* LSD region_grow's `cos(float(angle))` (lsd.cpp:678) resolved to the float
  overload: it calls sincosf (the seed's double std::cos: sincos).

/root/reference is absent on the GPU box: the module skips there.
"""
import collections
import pathlib
import re
import shutil
import struct
import subprocess

import pytest

REF = pathlib.Path("/root/reference")
MAIN = REF / "build/CMakeFiles/ORB_SLAM3-Relocalization.dir"
LINEDESC = REF / "Thirdparty/line_descriptor/build/CMakeFiles/linedesc.dir"

pytestmark = pytest.mark.skipif(not (MAIN / "src").is_dir() or shutil.which("objdump") is None,
                                reason="reference build tree / objdump not available")

FMA = re.compile(r"^vf(n)?m(add|sub)\d+[sp][sd]\b")

_cache = {}


def _disasm(obj):
    """{demangled function: [normalised instruction]}; a relocation's symbol is
    appended to its instruction as ' [sym]', branch / call addresses dropped."""
    obj = str(obj)
    if obj in _cache:
        return _cache[obj]
    out = subprocess.run(["objdump", "-dr", "--no-show-raw-insn", "-C", obj], capture_output=True, text=True,
                         check=True).stdout
    res, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            cur = m.group(1)
            res.setdefault(cur, [])
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+[0-9a-f]+: (R_X86_64_\w+)\s+(.*)$", line)
        if m:
            sym = re.sub(r"[-+]0x[0-9a-f]+$", "", m.group(2)).strip()
            res[cur][-1] += " [" + re.sub(r"\(.*$", "", sym) + "]"
            continue
        m = re.match(r"^\s+[0-9a-f]+:\t(.*)$", line)
        if m:
            ins = re.sub(r"\s+#.*$", "", m.group(1)).strip()
            ins = re.sub(r"\s+<.*>$", "", ins)
            ins = re.sub(r"\s+", " ", ins)
            ins = re.sub(r"^(call|j\w+) [0-9a-f]+", r"\1", ins)
            res[cur].append(ins)
    _cache[obj] = res
    return res


def _fn(obj, prefix):
    d = _disasm(obj)
    keys = [k for k in d if k.startswith(prefix) and "[clone" not in k]
    assert len(keys) == 1, (prefix, keys)
    return d[keys[0]]


def _fused(ins):
    return collections.Counter(s.split(" ")[0] for s in ins if FMA.match(s))


def _find(ins, pat, gap=8):
    """Number of places where `pat` occurs in order, each item within `gap`
    instructions of the previous one."""
    n = 0
    for i, s in enumerate(ins):
        if s != pat[0]:
            continue
        j, ok = i, True
        for p in pat[1:]:
            nxt = [k for k in range(j + 1, min(len(ins), j + 1 + gap)) if ins[k] == p]
            if not nxt:
                ok = False
                break
            j = nxt[0]
        n += ok
    return n


def _rodata(obj, sym, fmt):
    """Value of a local .rodata constant (.LCnn) of `obj`."""
    t = subprocess.run(["objdump", "-t", str(obj)], capture_output=True, text=True, check=True).stdout
    m = re.search(r"^([0-9a-f]+)\s+l\s+(\.rodata\S*)\s+[0-9a-f]+\s+" + re.escape(sym) + r"$", t, re.M)
    off, sec = int(m.group(1), 16), m.group(2)
    s = subprocess.run(["objdump", "-s", "-j", sec, str(obj)], capture_output=True, text=True, check=True).stdout
    data = bytearray()
    for line in s.splitlines():
        parts = line.split()
        if len(parts) > 1 and re.fullmatch(r"[0-9a-f]{4,}", parts[0]):
            for w in parts[1:5]:
                if re.fullmatch(r"[0-9a-f]{2,8}", w):
                    data += bytes.fromhex(w)
    return struct.unpack_from("<" + fmt, data, off)[0]


O_LSD = MAIN / "src/LSD/lsd.cpp.o"
O_ORB = MAIN / "src/ORBextractor.cc.o"
O_LEXT = MAIN / "src/LineExtractor.cc.o"
O_LM = MAIN / "src/LineMatcher.cpp.o"
O_OM = MAIN / "src/ORBmatcher.cc.o"
O_FR = MAIN / "src/Frame.cc.o"
O_KB8 = MAIN / "src/CameraModels/KannalaBrandt8.cpp.o"
O_PIN = MAIN / "src/CameraModels/Pinhole.cpp.o"
O_MP = MAIN / "src/MapPoint.cc.o"
O_TR = MAIN / "src/Tracking.cc.o"
O_GRID = MAIN / "src/gridStructure.cpp.o"
O_LIT = MAIN / "src/LineIterator.cpp.o"
O_LSDDET = LINEDESC / "src/LSDDetector_custom.cpp.o"
O_LBD = LINEDESC / "src/binary_descriptor_custom.cpp.o"


def test_compiler_and_flags():
    """GCC 9.4 for every path object (libstdc++ 9: the GCC <= 10 range-insert
    rule), the main library at -O3 -march=native (FMA contraction on), the
    line_descriptor library without -march (SSE2 only)."""
    for o in (O_LSD, O_ORB, O_LEXT, O_LM, O_OM, O_FR, O_KB8, O_GRID, O_LIT, O_LSDDET, O_LBD):
        c = subprocess.run(["readelf", "-p", ".comment", str(o)], capture_output=True, text=True, check=True).stdout
        assert "GCC: (Ubuntu 9.4.0-1ubuntu1~20.04.1) 9.4.0" in c, o
    main = (MAIN / "flags.make").read_text()
    assert re.search(r"CXX_FLAGS = .*-O3 -std=c\+\+11 .*-march=native", main)
    ld = (LINEDESC / "flags.make").read_text()
    assert re.search(r"CXX_FLAGS = .*-O3 -mtune=native", ld) and "-march" not in ld


def test_line_descriptor_is_plain_sse2():
    """LBD (binary_descriptor_custom.cpp) and KeyLine assembly
    (LSDDetector_custom.cpp): no fused op, no VEX instruction at all, and the
    float libm calls the oracle assumes."""
    for o in (O_LSDDET, O_LBD):
        for name, ins in _disasm(o).items():
            assert not [s for s in ins if s.startswith("v")], (o.name, name)
    und = lambda o: set(subprocess.run(["nm", "-u", str(o)], capture_output=True, text=True,  # noqa: E731
                                       check=True).stdout.split())
    assert {"cosf", "sinf", "roundf", "sqrtf", "exp"} <= und(O_LBD)
    assert {"atan2f", "sqrt", "pow"} <= und(O_LSDDET)


def test_float_overloads_on_the_path():
    """cos(float(angle)) in region_grow (lsd.cpp:678-679) is the float overload
    (sincosf), the seed's std::cos(double) (:648-649) the double one (sincos);
    computeOrbDescriptor's cos/sin of a float angle (ORBextractor.cc:111) is
    sincosf; KannalaBrandt8::project(Point3f) uses atan2f twice and sincosf."""
    rg = _fn(O_LSD, "cv::LineSegmentDetectorImpl::region_grow(")
    calls = [s for s in rg if s.startswith("call")]
    assert calls == ["call [sincos]", "call [sincosf]", "call [cv::fastAtan2]"]
    orb = _fn(O_ORB, "ORB_SLAM3::ORBextractor::operator()")
    assert "call [sincosf]" in orb and "call [sinf]" not in orb and "call [cosf]" not in orb
    kb = _fn(O_KB8, "ORB_SLAM3::KannalaBrandt8::project(cv::Point3_<float> const&)")
    # (sqrtf: the errno path of vsqrtss for a negative argument)
    assert [s for s in kb if s.startswith("call")] == ["call [atan2f]", "call [atan2f]", "call [sincosf]",
                                                        "call [sqrtf]"]


# every fused multiply-add in the path functions of the main library; any
# function of these objects not listed here (IC_Angle, DistributeOctTree,
# ComputePyramid, region_grow, SearchByBoW, SearchForInitialization, the
# local-map / relocalization SearchByProjection, LineMatcher::match /
# matchNNR / SearchByProjection, GetFeaturesInArea, AssignFeaturesToGrid,
# UndistortKeyPoints, ...) holds none (test_no_other_fused_ops)
FUSED = {
    (O_ORB, "ORB_SLAM3::ORBextractor::operator()"): {"vfmadd231ss": 16, "vfmsub132ss": 16},
    (O_LSD, "cv::LineSegmentDetectorImpl::ll_angle("): {"vfmadd231sd": 1},
    (O_LSD, "cv::LineSegmentDetectorImpl::flsd("): {"vfmadd213sd": 1},
    (O_LSD, "cv::LineSegmentDetectorImpl::get_theta("): {"vfmadd231sd": 2, "vfnmadd231sd": 1, "vfmadd132sd": 1},
    (O_LSD, "cv::LineSegmentDetectorImpl::region2rect("): {"vfmadd231sd": 3, "vfnmadd231sd": 1, "vfmadd132pd": 1},
    (O_LEXT, "ORB_SLAM3::Lineextractor::operator()"): {"vfmsub231sd": 1, "vfmadd132sd": 1},
    (O_LM, "ORB_SLAM3::LineMatcher::matchGrid("): {"vfmadd231sd": 2},
    (O_OM, "ORB_SLAM3::ORBmatcher::SearchByProjection(ORB_SLAM3::Frame&, ORB_SLAM3::Frame const&"):
        {"vfnmadd132ss": 1},
    (O_FR, "ORB_SLAM3::Frame::ComputeStereoMatches()"): {"vfmadd132ss": 1, "vfnmadd132ss": 1, "vfnmadd231ss": 1},
    (O_FR, "ORB_SLAM3::Frame::ComputeStereoMatches_Lines()"):
        {"vfmadd231sd": 2, "vfmsub231sd": 2, "vfmadd132sd": 2},
    (O_FR, "ORB_SLAM3::Frame::isInFrustum("): {"vfnmadd132ss": 1},
    (O_FR, "ORB_SLAM3::Frame::isInFrustum_l("): {"vfmadd213ss": 4},
    (O_KB8, "ORB_SLAM3::KannalaBrandt8::project(cv::Point3_<float> const&)"): {"vfmadd231ss": 1, "vfmadd132ss": 6},
}

# path functions whose objects hold fused ops elsewhere (control plane) but
# which themselves are one IEEE op per operator
UNFUSED = {
    O_LSD: ["cv::LineSegmentDetectorImpl::region_grow(", "cv::LineSegmentDetectorImpl::detect("],
    O_ORB: ["ORB_SLAM3::computeOrientation(", "ORB_SLAM3::ORBextractor::ComputePyramid(",
            "ORB_SLAM3::ORBextractor::ORBextractor(", "ORB_SLAM3::ORBextractor::DistributeOctTree(",
            "ORB_SLAM3::ORBextractor::ComputeKeyPointsOctTree("],
    O_OM: ["ORB_SLAM3::ORBmatcher::DescriptorDistance(",
           "ORB_SLAM3::ORBmatcher::SearchByProjection(ORB_SLAM3::Frame&, std::vector<",
           "ORB_SLAM3::ORBmatcher::SearchByProjection(ORB_SLAM3::Frame&, ORB_SLAM3::KeyFrame*",
           "ORB_SLAM3::ORBmatcher::SearchByBoW(ORB_SLAM3::KeyFrame*, ORB_SLAM3::Frame&",
           "ORB_SLAM3::ORBmatcher::SearchForInitialization("],
    O_LM: ["ORB_SLAM3::LineMatcher::SearchByProjection(", "ORB_SLAM3::LineMatcher::matchNNR(",
           "ORB_SLAM3::LineMatcher::match(cv::Mat", "ORB_SLAM3::LineMatcher::SerachForInitialize("],
    O_FR: ["ORB_SLAM3::Frame::GetFeaturesInArea(", "ORB_SLAM3::Frame::PosInGrid(", "ORB_SLAM3::Frame::AssignFeaturesToGrid(",
           "ORB_SLAM3::Frame::UndistortKeyPoints(", "ORB_SLAM3::Frame::UndistortKeyLines(",
           "ORB_SLAM3::Frame::ComputeImageBounds(", "ORB_SLAM3::Frame::ComputeBoW(",
           "ORB_SLAM3::Frame::lineDescriptorMAD(", "ORB_SLAM3::Frame::isInFrustumChecks("],
    O_PIN: ["ORB_SLAM3::Pinhole::project(cv::Point3_<float> const&)"],
    O_MP: ["ORB_SLAM3::MapPoint::PredictScale(float const&, ORB_SLAM3::Frame*)",
           "ORB_SLAM3::MapPoint::GetMinDistanceInvariance(", "ORB_SLAM3::MapPoint::GetMaxDistanceInvariance("],
    O_TR: ["ORB_SLAM3::Tracking::SearchLocalPointsAndLines("],
    O_GRID: ["ORB_SLAM3::GridStructure::get(", "ORB_SLAM3::getLineCoords("],
    O_LIT: ["ORB_SLAM3::LineIterator::LineIterator(", "ORB_SLAM3::LineIterator::getNext("],
}


@pytest.mark.parametrize("key", list(FUSED), ids=[k[1].split("(")[0].split("::")[-1] + "@" + k[0].name
                                                  for k in FUSED])
def test_fused_ops_per_function(key):
    assert _fused(_fn(*key)) == collections.Counter(FUSED[key])


def test_no_other_fused_ops():
    for obj, names in UNFUSED.items():
        for n in names:
            assert not _fused(_fn(obj, n)), (obj.name, n)
    # ORBextractor.cc.o: the descriptor's 32 are all there is
    assert sum(sum(_fused(v).values()) for v in _disasm(O_ORB).values()) == 32


def test_orb_descriptor_sample_positions():
    """computeOrbDescriptor (ORBextractor.cc:116-118, inlined into operator()):
    a = cos -> xmm1, b = sin -> xmm0 (sincosf(angle, &sin=-0x404, &cos=-0x408));
    per sample y*a and y*b are rounded, then row = fma(x, b, y*a) and
    col = fma(x, a, -(y*b))."""
    f = _fn(O_ORB, "ORB_SLAM3::ORBextractor::operator()")
    assert _find(f, ["lea -0x404(%rbp),%rax", "mov %rax,-0x470(%rbp)", "lea -0x408(%rbp),%rax",
                     "mov %rax,-0x440(%rbp)"]) == 1
    assert _find(f, ["mov -0x440(%rbp),%rsi", "mov -0x470(%rbp),%rdi", "call [sincosf]",
                     "vmovss -0x408(%rbp),%xmm1", "vmovss -0x404(%rbp),%xmm0"]) == 1
    assert _find(f, ["vcvtsi2ssl 0x4(%r12),%xmm5,%xmm4", "vcvtsi2ssl (%r12),%xmm5,%xmm3", "vmulss %xmm4,%xmm1,%xmm2",
                     "vmulss %xmm4,%xmm0,%xmm4", "vfmadd231ss %xmm3,%xmm0,%xmm2", "vfmsub132ss %xmm1,%xmm4,%xmm3",
                     "vcvtss2si %xmm2,%esi"], gap=1) == 1
    assert _find(f, ["vmulss %xmm3,%xmm1,%xmm4", "vmulss %xmm3,%xmm0,%xmm3", "vfmadd231ss %xmm2,%xmm0,%xmm4",
                     "vfmsub132ss %xmm1,%xmm3,%xmm2"], gap=6) == 15


def test_lsd_fused_sites():
    """ll_angle (lsd.cpp:565-569): norm = sqrt(fma(gx, gx, gy*gy) * 0.25);
    get_theta (:754-770): Ixx = fma(dy*dy, w, Ixx), Iyy = fma(dx*dx, w, Iyy),
    Ixy = Ixy - (dx*dy)*w fused, lambda's root of fma(d, d, (4*Ixy)*Ixy);
    region2rect (:692-733): x = fma(x_i, w, x), y = fma(y_i, w, y),
    l = fma(regdx, dx, regdy*dy), the four endpoints fma(l, d, c) in one
    vfmadd132pd; flsd's LOG_NT = fma(5*(lw + lh), 0.5, log10(11.0) as folded
    by GCC)."""
    la = _fn(O_LSD, "cv::LineSegmentDetectorImpl::ll_angle(")
    assert _find(la, ["vaddsd %xmm0,%xmm1,%xmm2", "vsubsd %xmm0,%xmm1,%xmm1", "vmulsd %xmm1,%xmm1,%xmm0",
                      "vfmadd231sd %xmm2,%xmm2,%xmm0", "vmulsd %xmm4,%xmm0,%xmm0", "vsqrtsd %xmm0,%xmm0,%xmm5"],
                 gap=3) == 1
    gt = _fn(O_LSD, "cv::LineSegmentDetectorImpl::get_theta(")
    assert _find(gt, ["vsubsd %xmm8,%xmm2,%xmm2", "vsubsd %xmm9,%xmm0,%xmm0", "vmulsd %xmm2,%xmm2,%xmm7",
                      "vfmadd231sd %xmm3,%xmm7,%xmm4", "vmulsd %xmm0,%xmm0,%xmm7", "vmulsd %xmm2,%xmm0,%xmm0",
                      "vfmadd231sd %xmm7,%xmm3,%xmm5", "vfnmadd231sd %xmm0,%xmm3,%xmm1"], gap=1) == 1
    assert _find(gt, ["vmulsd 0x0(%rip),%xmm1,%xmm7 [.LC42]", "vsubsd %xmm5,%xmm4,%xmm0", "vaddsd %xmm5,%xmm4,%xmm2",
                      "vmulsd %xmm1,%xmm7,%xmm7", "vfmadd132sd %xmm0,%xmm7,%xmm0", "vsqrtsd %xmm0,%xmm0,%xmm7"],
                 gap=3) == 1
    assert _rodata(O_LSD, ".LC42", "d") == 4.0
    rr = _fn(O_LSD, "cv::LineSegmentDetectorImpl::region2rect(")
    assert _find(rr, ["vcvtsi2sdl (%rax),%xmm4,%xmm1", "vmovsd 0x18(%rax),%xmm0", "add $0x20,%rax",
                      "vaddsd %xmm0,%xmm6,%xmm6", "vfmadd231sd %xmm0,%xmm1,%xmm5", "vcvtsi2sdl -0x1c(%rax),%xmm4,%xmm1",
                      "vfmadd231sd %xmm1,%xmm0,%xmm3"], gap=1) == 1
    assert _find(rr, ["lea -0x90(%rbp),%rdi", "lea -0x98(%rbp),%rsi", "call [sincos]", "vmovsd -0x98(%rbp),%xmm6",
                      "vmovsd -0x90(%rbp),%xmm5"]) == 1  # dx = cos -> xmm6, dy = sin -> xmm5
    assert _find(rr, ["vsubsd %xmm11,%xmm3,%xmm3", "vsubsd %xmm12,%xmm1,%xmm1", "vmulsd %xmm3,%xmm5,%xmm13",
                      "vmulsd %xmm3,%xmm6,%xmm3", "vfmadd231sd %xmm1,%xmm6,%xmm13", "vfnmadd231sd %xmm5,%xmm1,%xmm3"],
                 gap=1) == 1
    assert _find(rr, ["vfmadd132pd %ymm10,%ymm1,%ymm8"]) == 1
    fl = _fn(O_LSD, "cv::LineSegmentDetectorImpl::flsd(")
    assert _find(fl, ["call [log10]", "call [log10]", "vaddsd -0x2f8(%rbp),%xmm0,%xmm1",
                      "vmulsd 0x0(%rip),%xmm1,%xmm1 [.LC73]", "vmovsd 0x0(%rip),%xmm5 [.LC43]",
                      "vfmadd213sd 0x0(%rip),%xmm5,%xmm1 [.LC74]"], gap=6) == 1
    assert (_rodata(O_LSD, ".LC73", "d"), _rodata(O_LSD, ".LC43", "d")) == (5.0, 0.5)
    assert _rodata(O_LSD, ".LC74", "d").hex() == "0x1.0a98b6050c56fp+0"  # oracle/lines_oracle.cpp, kLog10Of11


def test_line_fused_sites():
    """Lineextractor::operator() lineFns (LineExtractor.cc:106-111): c =
    fma(sx, ey, -(sy*ex)), norm = sqrt(fma(a, a, b*b)); matchGrid
    (LineMatcher.cpp:221-231, normalize / dot of LineMatcher.h): sqrt(fma(vx,
    vx, vy*vy)) and fma(vx, d.x, vy*d.y)."""
    le = _fn(O_LEXT, "ORB_SLAM3::Lineextractor::operator()")
    assert _find(le, ["vcvtss2sd 0x1c(%rbx),%xmm5,%xmm0", "vmovapd %xmm0,%xmm2", "vcvtss2sd 0x20(%rbx),%xmm5,%xmm1",
                      "vcvtss2sd 0x24(%rbx),%xmm5,%xmm0", "vcvtss2sd 0x28(%rbx),%xmm5,%xmm3", "vmulsd %xmm0,%xmm1,%xmm4",
                      "vsubsd %xmm3,%xmm1,%xmm1", "vsubsd %xmm2,%xmm0,%xmm0", "vfmsub231sd %xmm3,%xmm2,%xmm4",
                      "vmulsd %xmm1,%xmm1,%xmm1", "vfmadd132sd %xmm0,%xmm1,%xmm0", "vsqrtsd %xmm0,%xmm0,%xmm1"],
                 gap=5) == 1
    mg = _fn(O_LM, "ORB_SLAM3::LineMatcher::matchGrid(")
    assert _find(mg, ["vmulsd %xmm0,%xmm0,%xmm0", "vfmadd231sd %xmm1,%xmm1,%xmm0"], gap=1) == 1
    assert _find(mg, ["vmulsd 0x8(%rdx),%xmm2,%xmm0", "vfmadd231sd (%rdx),%xmm3,%xmm0"], gap=1) == 1


def test_projection_and_stereo_fused_sites():
    """SearchByProjection(F, F) (ORBmatcher.cc:2043): ur = uv.x - mbf*invzc
    fused; KannalaBrandt8::project(Point3f) (KannalaBrandt8.cpp:29-42): x*x +
    y*y, the four r terms, u and v fused; ComputeStereoMatches
    (Frame.cc:1249-1251, :1367): kpY +/- 2*scale and dist1 + dist3 -
    2*dist2 fused; ComputeStereoMatches_Lines (:1437, :1464, :1469-1470,
    :1489): normalize, the crosses, the endpoint re-projection."""
    sb = _fn(O_OM, "ORB_SLAM3::ORBmatcher::SearchByProjection(ORB_SLAM3::Frame&, ORB_SLAM3::Frame const&")
    assert _find(sb, ["vfnmadd132ss 0x1c0(%rsi),%xmm7,%xmm0", "vsubss %xmm1,%xmm0,%xmm0"], gap=1) == 1
    kb = _fn(O_KB8, "ORB_SLAM3::KannalaBrandt8::project(cv::Point3_<float> const&)")
    assert _find(kb, ["vmovss 0x4(%rdx),%xmm1", "vmovss (%rdx),%xmm0", "vmulss %xmm1,%xmm1,%xmm1",
                      "vfmadd132ss %xmm0,%xmm1,%xmm0"], gap=1) == 1
    assert _find(kb, ["vmulss %xmm2,%xmm2,%xmm0", "vmovss 0xc(%rdx),%xmm5", "vmovss 0x8(%rdx),%xmm6",
                      "vmulss %xmm0,%xmm2,%xmm4", "vfmadd231ss 0x10(%rdx),%xmm4,%xmm2", "vmulss %xmm4,%xmm0,%xmm3",
                      "vmulss %xmm3,%xmm0,%xmm1", "vfmadd132ss 0x14(%rdx),%xmm2,%xmm3", "vmulss %xmm1,%xmm0,%xmm0",
                      "vfmadd132ss 0x18(%rdx),%xmm3,%xmm1", "vfmadd132ss 0x1c(%rdx),%xmm1,%xmm0",
                      "vmulss 0x4(%rdx),%xmm0,%xmm1", "vmulss (%rdx),%xmm0,%xmm0", "vfmadd132ss 0xc(%rsp),%xmm5,%xmm1",
                      "vfmadd132ss 0x8(%rsp),%xmm6,%xmm0"], gap=1) == 1
    cs = _fn(O_FR, "ORB_SLAM3::Frame::ComputeStereoMatches()")
    assert _find(cs, ["vfmadd132ss %xmm0,%xmm2,%xmm1", "vfnmadd132ss 0x0(%rip),%xmm2,%xmm0 [.LC72]",
                      "vroundss $0xa,%xmm1,%xmm1,%xmm1", "vroundss $0x9,%xmm0,%xmm0,%xmm0"], gap=1) == 1
    assert _find(cs, ["vsubss %xmm2,%xmm0,%xmm1", "vaddss %xmm2,%xmm0,%xmm0",
                      "vfnmadd231ss 0x0(%rip),%xmm3,%xmm0 [.LC72]", "vaddss %xmm0,%xmm0,%xmm0",
                      "vdivss %xmm0,%xmm1,%xmm1"], gap=2) == 1
    assert _rodata(O_FR, ".LC72", "f") == 2.0
    cl = _fn(O_FR, "ORB_SLAM3::Frame::ComputeStereoMatches_Lines()")
    assert _find(cl, ["vmulsd %xmm5,%xmm5,%xmm8", "vmovsd %xmm5,0x8(%rbx)", "vmovsd %xmm4,(%rbx)",
                      "vfmadd231sd %xmm4,%xmm4,%xmm8"], gap=1) == 1
    # sp_r / ep_r re-projection: xmm4 = sp_l(1), xmm10 = ep_l(1), xmm2 = sp_r(1),
    # xmm7 = ep_r(1), xmm5 = ep_r(0), -0x260 = sp_r(0), -0x280 = sp_r(1) - ep_r(1)
    assert _find(cl, ["vsubsd %xmm4,%xmm2,%xmm0", "vsubsd %xmm10,%xmm4,%xmm2", "vsubsd %xmm7,%xmm10,%xmm1",
                      "vsubsd %xmm7,%xmm4,%xmm3", "vmulsd %xmm5,%xmm2,%xmm2", "vmulsd %xmm5,%xmm0,%xmm0",
                      "vfmadd231sd -0x260(%rbp),%xmm3,%xmm0", "vdivsd -0x280(%rbp),%xmm0,%xmm0",
                      "vfmadd132sd %xmm1,%xmm2,%xmm0"], gap=6) == 1
    assert _find(cl, ["vmulsd %xmm0,%xmm1,%xmm5", "vsubsd %xmm2,%xmm0,%xmm0", "vsubsd %xmm4,%xmm1,%xmm1",
                      "vfmsub231sd %xmm4,%xmm2,%xmm5", "vmulsd %xmm1,%xmm1,%xmm1", "vfmadd132sd %xmm0,%xmm1,%xmm0",
                      "vsqrtsd %xmm0,%xmm0,%xmm1"], gap=6) == 1


def test_frustum_sites():
    """Frame::isInFrustum (Frame.cc:777, :810, :823): invz = 1.0f/PcZ, viewCos
    = (float)(PO.dot(Pn) / (double)dist), mTrackProjXR = fma(-mbf, invz, u);
    isInFrustum_l (:871-873, :895-897, :930): u = fma(fx*PcX, invz, cx) per
    coordinate, mnTrackangle = (double)atan2f(eY - sY, eX - sX);
    MapPoint::PredictScale (MapPoint.cc:539-545): logf, a float division,
    ceil (vroundss $0xa), cvttss2si, the clamp (negative -> 0 first); the
    line filter of SearchLocalPointsAndLines calls atan2f (Tracking.cc:5260)."""
    fr = _fn(O_FR, "ORB_SLAM3::Frame::isInFrustum(")
    assert _find(fr, ["vdivss -0x408(%rbp),%xmm0,%xmm0", "vmovss -0x420(%rbp),%xmm7", "vmovss %xmm1,0x1c(%rbx)",
                      "vfnmadd132ss 0x1c0(%r12),%xmm1,%xmm0"], gap=3) == 1
    assert _find(fr, ["vcvtss2sd -0x3fc(%rbp),%xmm0,%xmm0", "vdivsd %xmm0,%xmm1,%xmm0",
                      "vcvtsd2ss %xmm0,%xmm0,%xmm6"], gap=1) == 1
    calls = [c for c in fr if c.startswith("call [") and c.split("[")[1].rstrip("]") in (
        "cv::norm", "cv::Mat::dot", "ORB_SLAM3::MapPoint::PredictScale", "cv::operator*", "cv::operator+",
        "cv::operator-")]
    assert calls == ["call [cv::operator*]", "call [cv::operator+]", "call [cv::norm]", "call [cv::operator-]",
                     "call [cv::norm]", "call [cv::Mat::dot]", "call [ORB_SLAM3::MapPoint::PredictScale]"]
    fl = _fn(O_FR, "ORB_SLAM3::Frame::isInFrustum_l(")
    for c in ("cx", "cy"):
        reg = "%xmm0" if c == "cx" else "%xmm2"
        acc = "%xmm1,%xmm0" if c == "cx" else "%xmm2,%xmm1"
        assert _find(fl, ["vmulss (%rax)," + reg + "," + reg, "mov 0x0(%rip),%rax [ORB_SLAM3::Frame::" + c + "]",
                          "vfmadd213ss (%rax)," + acc], gap=1) == 2
    assert _find(fl, ["vsubss 0x68(%r14),%xmm0,%xmm0", "vsubss 0x64(%r14),%xmm1,%xmm1", "call [atan2f]",
                      "vcvtss2sd %xmm0,%xmm0,%xmm0"], gap=1) == 1
    assert _find(fl, ["vcvtss2sd -0x4e8(%rbp),%xmm0,%xmm0", "vmovss -0x50c(%rbp),%xmm7", "vdivsd %xmm0,%xmm1,%xmm0",
                      "vcvtsd2ss %xmm0,%xmm0,%xmm0"], gap=1) == 1
    ps = _fn(O_MP, "ORB_SLAM3::MapPoint::PredictScale(float const&, ORB_SLAM3::Frame*)")
    assert _find(ps, ["call [logf]", "vdivss 0x129b8(%rbp),%xmm0,%xmm0", "vroundss $0xa,%xmm0,%xmm0,%xmm0",
                      "vcvttss2si %xmm0,%eax", "test %eax,%eax", "js"], gap=1) == 1
    assert _find(ps, ["cmp %eax,%edx", "lea -0x1(%rdx),%ecx", "cmovle %ecx,%eax"], gap=1) == 1
    assert "call [atan2f]" in _fn(O_TR, "ORB_SLAM3::Tracking::SearchLocalPointsAndLines(")
    for name, want in (("GetMinDistanceInvariance", 0.8), ("GetMaxDistanceInvariance", 1.2)):
        f = _fn(O_MP, "ORB_SLAM3::MapPoint::" + name + "(")
        lc = [re.search(r"\[(\.LC\d+)\]", s).group(1) for s in f if s.startswith("vmovss 0x0(%rip)")]
        assert len(lc) == 1 and any(s.startswith("vmulss") for s in f), name
        assert _rodata(O_MP, lc[0], "f") == struct.unpack("<f", struct.pack("<f", want))[0], name


def test_grid_get_passes_the_range_length_as_rehash_hint():
    """GridStructure::get (gridStructure.cpp:67-78) as libstdc++ 9 inlines
    indices.insert(first, last): n_elt = list size, `if (n_elt != 1) --n_elt`
    for a key already present, n_elt handed to _M_need_rehash -- the GCC <= 10
    rule the product emulates by default (csrc/stl_uset.h range_hint=1; GCC 11
    passes 1)."""
    g = _fn(O_GRID, "ORB_SLAM3::GridStructure::get(")
    assert _find(g, ["mov 0x10(%rbp),%r14", "cmp $0x1,%r14", "setne %al", "sub %rax,%r14"], gap=40) == 1
    assert _find(g, ["mov %r14,%rcx", "call [std::__detail::_Prime_rehash_policy::_M_need_rehash]"], gap=12) == 1
