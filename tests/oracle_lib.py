"""ctypes loader for the CPU oracle (oracle/, test infrastructure only).

Builds oracle/_build/liboracle.so with `make -C oracle` when missing.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this.
"""
import ctypes
import os
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
LIB = ORACLE_DIR / "_build" / "liboracle.so"
# ORACLE_LIB: another build of the same sources (bench.py's -march=native CPU baseline)
LIB_OVERRIDE = os.environ.get("ORACLE_LIB")


class KP(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float), ("angle", ctypes.c_float),
                ("response", ctypes.c_float), ("octave", ctypes.c_int), ("class_id", ctypes.c_int)]


KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    srcs = list(ORACLE_DIR.glob("*.cpp")) + list(ORACLE_DIR.glob("*.h")) + list(ORACLE_DIR.glob("*.inc"))
    if LIB_OVERRIDE:
        lib = ctypes.CDLL(LIB_OVERRIDE)
    else:
        if not LIB.exists() or any(s.stat().st_mtime > LIB.stat().st_mtime for s in srcs):
            build()
        lib = ctypes.CDLL(str(LIB))
    V, I, F, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
    P = ctypes.POINTER(ctypes.c_int)
    lib.oracle_orb_extract.argtypes = [V, I, I, I, I, F, I, I, I, I, I, V, V, I, P]
    lib.oracle_orb_extract.restype = I
    lib.oracle_orb_stage.argtypes = [V, I, I, I, F, I, I, I, I, V, V, P, P, V, I, P, V, I, P]
    lib.oracle_orb_stage.restype = I
    lib.oracle_orb_params.argtypes = [I, F, I, V, V, V]
    lib.oracle_resize_u8.argtypes = [V, I, I, V, I, I]
    lib.oracle_gaussian_blur_u8.argtypes = [V, I, I, I, D, V]
    lib.oracle_gaussian_taps_u8.argtypes = [I, D, V]
    lib.oracle_gaussian_kernel_f64.argtypes = [I, D, V]
    lib.oracle_fast_atan2.argtypes = [F, F]
    lib.oracle_fast_atan2.restype = F
    lib.oracle_search_by_bow.argtypes = [V, V, V, V, V, I, V, V, V, I, V, V, I, V, F, I, V]
    lib.oracle_search_by_bow.restype = I
    lib.oracle_descriptor_distance.argtypes = [V, V]
    lib.oracle_descriptor_distance.restype = I
    lib.oracle_line_descriptor_distance.argtypes = [V, V]
    lib.oracle_line_descriptor_distance.restype = I
    lib.oracle_match_grid.argtypes = [V, V, I, I, I, V, V, V, V, I, I, I, I, I, V]
    lib.oracle_match_grid.restype = I
    lib.oracle_match_grid2.argtypes = [V, V, I, I, I, V, V, V, V, I, I, I, I, I, I, V]
    lib.oracle_match_grid2.restype = I
    lib.oracle_uset_order.argtypes = [V, V, I, I, V]
    lib.oracle_uset_order.restype = I
    lib.oracle_grid_candidates.argtypes = [I, I, V, V, I, I, I, I, I, I, I, I, I, V, I]
    lib.oracle_grid_candidates.restype = I
    lib.oracle_line_coords.argtypes = [D, D, D, D, V, I]
    lib.oracle_line_coords.restype = I
    lib.oracle_fast_score.argtypes = [V, I]
    lib.oracle_fast_score.restype = I
    lib.oracle_set_compat.argtypes = [ctypes.c_uint]
    lib.oracle_get_compat.restype = ctypes.c_uint
    lib.oracle_cv_exp_table.argtypes = [D]
    lib.oracle_cv_exp_table.restype = D
    lib.oracle_match_nnr_inout.argtypes = [V, I, V, I, F, V, I]
    lib.oracle_match_nnr_inout.restype = I
    lib.oracle_match_inout.argtypes = [V, I, V, I, F, V, I]
    lib.oracle_match_inout.restype = I
    _lib = lib
    return lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


class compat:
    """with compat(bits): run the oracle under the PLVI_COMPAT_* switches."""

    def __init__(self, bits):
        self.bits = bits

    def __enter__(self):
        lib = load()
        self.prev = lib.oracle_get_compat()
        lib.oracle_set_compat(self.bits)
        return self

    def __exit__(self, *exc):
        load().oracle_set_compat(self.prev)
        return False


def cv_exp_table(x):
    return load().oracle_cv_exp_table(float(x))


def orb_extract(img, nfeatures=1000, scale=1.2, nlevels=8, ini=20, mn=7, lap=(0, 0), cap=20000):
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int()
    mono = lib.oracle_orb_extract(_p(img), w, h, w, nfeatures, scale, nlevels, ini, mn, lap[0], lap[1],
                                  _p(kps), _p(desc), cap, ctypes.byref(n))
    return mono, kps[:n.value].copy(), desc[:n.value].copy()


def orb_stage(img, level, nfeatures=1000, scale=1.2, nlevels=8, ini=20, mn=7, cap=200000):
    lib = load()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    pyr = np.zeros(w * h, np.uint8)
    blur = np.zeros(w * h, np.uint8)
    lw, lh, nc, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    cand = np.zeros((cap, 3), np.float32)
    lvk = np.zeros((cap, 4), np.float32)
    rc = lib.oracle_orb_stage(_p(img), w, h, nfeatures, scale, nlevels, ini, mn, level, _p(pyr), _p(blur),
                              ctypes.byref(lw), ctypes.byref(lh), _p(cand), cap, ctypes.byref(nc), _p(lvk), cap,
                              ctypes.byref(nl))
    assert rc == 0
    n = lw.value * lh.value
    return {"pyr": pyr[:n].reshape(lh.value, lw.value), "blur": blur[:n].reshape(lh.value, lw.value),
            "cand": cand[:nc.value], "levelkps": lvk[:nl.value]}


def resize(src, dw, dh):
    lib = load()
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib.oracle_resize_u8(_p(src), src.shape[1], src.shape[0], _p(out), dw, dh)
    return out


def gaussian_blur(src, ksize, sigma):
    lib = load()
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros_like(src)
    lib.oracle_gaussian_blur_u8(_p(src), src.shape[1], src.shape[0], ksize, sigma, _p(out))
    return out


def gaussian_taps(ksize, sigma):
    lib = load()
    t = np.zeros(ksize, np.int32)
    lib.oracle_gaussian_taps_u8(ksize, sigma, _p(t))
    return t


def gaussian_kernel_f64(ksize, sigma):
    lib = load()
    t = np.zeros(ksize, np.float64)
    lib.oracle_gaussian_kernel_f64(ksize, sigma, _p(t))
    return t


def _declare_match(lib):
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_knn2.argtypes = [V, I, V, I, V, V, V, V]
    lib.oracle_match_nnr.argtypes = [V, I, V, I, F, V]
    lib.oracle_match_nnr.restype = I
    lib.oracle_match.argtypes = [V, I, V, I, F, V]
    lib.oracle_match.restype = I
    lib.oracle_descriptor_distance.argtypes = [V, V]
    lib.oracle_line_descriptor_distance.argtypes = [V, V]


def knn2(q, t):
    lib = load()
    _declare_match(lib)
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    out = [np.zeros(q.shape[0], np.int32) for _ in range(4)]
    lib.oracle_knn2(_p(q), q.shape[0], _p(t), t.shape[0], *[_p(o) for o in out])
    return tuple(out)


def _match_inout(fn, d1, d2, nnr, prev):
    d1 = np.ascontiguousarray(d1, np.uint8).reshape(-1, 32)
    d2 = np.ascontiguousarray(d2, np.uint8).reshape(-1, 32)
    prev = np.zeros(0, np.int32) if prev is None else np.ascontiguousarray(prev, np.int32)
    m = np.full(max(d1.shape[0], prev.size, 1), -1, np.int32)
    m[:prev.size] = prev
    n = fn(_p(d1), d1.shape[0], _p(d2), d2.shape[0], nnr, _p(m), prev.size)
    return n, m[:d1.shape[0]].copy()


def match_nnr(d1, d2, nnr, prev=None):
    """LineMatcher::matchNNR; prev = the caller's existing matches_12 (kept by resize)."""
    return _match_inout(load().oracle_match_nnr_inout, d1, d2, nnr, prev)


def match(d1, d2, nnr, prev=None):
    """LineMatcher::match (mutual); returns -2 for a stale out-of-range entry (UB in the reference)."""
    return _match_inout(load().oracle_match_inout, d1, d2, nnr, prev)


KEYLINE_DTYPE = np.dtype([("angle", "<f4"), ("class_id", "<i4"), ("octave", "<i4"), ("pt_x", "<f4"),
                          ("pt_y", "<f4"), ("response", "<f4"), ("size", "<f4"), ("startPointX", "<f4"),
                          ("startPointY", "<f4"), ("endPointX", "<f4"), ("endPointY", "<f4"),
                          ("sPointInOctaveX", "<f4"), ("sPointInOctaveY", "<f4"), ("ePointInOctaveX", "<f4"),
                          ("ePointInOctaveY", "<f4"), ("lineLength", "<f4"), ("numOfPixels", "<i4")])


def line_extract(img, nfeatures=200, lsd_scale=0.8, nlevels=2, scale=2.0, cap=20000):
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_line_extract.argtypes = [V, I, I, I, I, F, I, F, V, V, V, I, ctypes.POINTER(I)]
    lib.oracle_line_extract.restype = I
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    kl = np.zeros(cap, KEYLINE_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    fn = np.zeros((cap, 3), np.float64)
    n = ctypes.c_int()
    rc = lib.oracle_line_extract(_p(img), w, h, w, nfeatures, lsd_scale, nlevels, scale, _p(kl), _p(desc), _p(fn),
                                 cap, ctypes.byref(n))
    assert rc == 0, rc
    k = n.value
    return kl[:k].copy(), desc[:k].copy(), fn[:k].copy()


def lsd_raw(img, lsd_scale=0.8, cap=20000):
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_lsd_raw.argtypes = [V, I, I, F, V, I, ctypes.POINTER(I)]
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros((cap, 4), np.float32)
    n = ctypes.c_int()
    lib.oracle_lsd_raw(_p(img), img.shape[1], img.shape[0], lsd_scale, _p(out), cap, ctypes.byref(n))
    return out[:n.value].copy()


def lsd_planes(img, lsd_scale=0.8):
    """flsd's scaled image, angle (rad, NOTDEF -1024) and modgrad planes (f64)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_lsd_planes.argtypes = [V, I, I, F, V, V, V, ctypes.POINTER(I), ctypes.POINTER(I)]
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    n = (w + 2) * (h + 2)
    bufs = [np.zeros(n, np.float64) for _ in range(3)]
    sw, sh = ctypes.c_int(), ctypes.c_int()
    rc = lib.oracle_lsd_planes(_p(img), w, h, lsd_scale, *[_p(b) for b in bufs], ctypes.byref(sw), ctypes.byref(sh))
    assert rc == 0, rc
    m = sw.value * sh.value
    return tuple(b[:m].reshape(sh.value, sw.value).copy() for b in bufs)


def lbd_sobel(img, octave):
    """LBD octave `octave` Sobel planes (dx, dy) int16 of computeGaussianPyramid + Sobel."""
    lib = load()
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.oracle_lbd_sobel.argtypes = [V, I, I, I, V, V, ctypes.POINTER(I), ctypes.POINTER(I)]
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    dx = np.zeros(w * h, np.int16)
    dy = np.zeros(w * h, np.int16)
    ow, oh = ctypes.c_int(), ctypes.c_int()
    assert lib.oracle_lbd_sobel(_p(img), w, h, octave, _p(dx), _p(dy), ctypes.byref(ow), ctypes.byref(oh)) == 0
    n = ow.value * oh.value
    return dx[:n].reshape(oh.value, ow.value), dy[:n].reshape(oh.value, ow.value)


def line_iterator_count(W, H, x1, y1, x2, y2):
    lib = load()
    F, I = ctypes.c_float, ctypes.c_int
    lib.oracle_line_iterator_count.argtypes = [I, I, F, F, F, F]
    return lib.oracle_line_iterator_count(W, H, x1, y1, x2, y2)


def search_by_bow(kf_desc, kf_angle, kf_live, kf_fv, f_desc, f_angle, f_fv, nnratio, check_orientation=True,
                  f_nleft=-1):
    """ORBmatcher::SearchByBoW restatement; fv = dict {node: [indices]}; f_nleft = F.Nleft (-1: one camera)."""
    lib = load()
    def csr(fv):
        nodes = np.array(sorted(fv), dtype=np.int32)
        off = np.zeros(len(nodes) + 1, np.int32)
        idx = []
        for i, n in enumerate(nodes):
            idx.extend(fv[int(n)])
            off[i + 1] = len(idx)
        return nodes, off, np.array(idx if idx else [0], dtype=np.int32)
    kn, ko, ki = csr(kf_fv)
    fn, fo, fi = csr(f_fv)
    kd = np.ascontiguousarray(kf_desc, np.uint8); ka = np.ascontiguousarray(kf_angle, np.float32)
    kl = np.ascontiguousarray(kf_live, np.uint8); fd = np.ascontiguousarray(f_desc, np.uint8)
    fa = np.ascontiguousarray(f_angle, np.float32)
    out = np.full(max(len(fd), 1), -1, np.int32)
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_by_bow2.argtypes = [V, V, V, V, V, I, V, V, V, I, V, V, I, V, F, I, I, V]
    lib.oracle_search_by_bow2.restype = I
    n = lib.oracle_search_by_bow2(_p(kd), _p(ka), _p(kl), _p(kn), _p(ko), len(kn), _p(ki), _p(fd), _p(fa), len(fd),
                                  _p(fn), _p(fo), len(fn), _p(fi), float(nnratio), int(check_orientation),
                                  int(f_nleft), _p(out))
    return n, out[:len(fd)]


def uset_order(cells, range_hint):
    """Iteration order of a std::unordered_set<int> filled by one range insert per cell list."""
    off = np.zeros(len(cells) + 1, np.int32)
    flat = []
    for i, c in enumerate(cells):
        flat.extend(c)
        off[i + 1] = len(flat)
    seq = np.array(flat if flat else [0], np.int32)
    out = np.zeros(max(len(flat), 1), np.int32)
    n = load().oracle_uset_order(_p(off), _p(seq), len(cells), range_hint, _p(out))
    return out[:n].tolist()


def match_grid(lines1, desc1, grid, desc2, directions2, window=((7, 0), (2, 2)), range_hint=0):
    """LineMatcher::matchGrid restatement (real std::unordered_set of the host libstdc++;
    range_hint=1 drives it with the GCC <= 10 range-insert hint, see match_oracle.cpp)."""
    lib = load()
    cols, rows = len(grid), len(grid[0])
    off = np.zeros(cols * rows + 1, np.int32)
    idx = []
    for x in range(cols):
        for y in range(rows):
            idx.extend(grid[x][y])
            off[x * rows + y + 1] = len(idx)
    idx = np.array(idx if idx else [0], np.int32)
    l1 = np.ascontiguousarray(lines1, np.int32).reshape(-1, 4)
    d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
    d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
    v2 = np.ascontiguousarray(directions2, np.float64).reshape(-1, 2)
    m = np.full(max(len(l1), 1), -1, np.int32)
    (w0, w1), (h0, h1) = window
    n = lib.oracle_match_grid2(_p(l1), _p(d1), len(l1), cols, rows, _p(off), _p(idx), _p(d2), _p(v2), len(d2),
                               w0, w1, h0, h1, range_hint, _p(m))
    return n, m[:len(l1)]


def _grid_csr(grid):
    cols, rows = len(grid), len(grid[0])
    off = np.zeros(cols * rows + 1, np.int32)
    idx = []
    for x in range(cols):
        for y in range(rows):
            idx.extend(grid[x][y])
            off[x * rows + y + 1] = len(idx)
    return cols, rows, off, np.array(idx if idx else [0], np.int32)


def grid_candidates(grid, sp, ep, window=((7, 0), (2, 2)), range_hint=0, lib=None, fn="oracle_grid_candidates"):
    """Iteration order of matchGrid's candidate set for one line (GridStructure::get
    at sp then ep, gridStructure.cpp:67-78).  `lib`/`fn` select another
    implementation with the same signature minus range_hint (oracle/_ref)."""
    cols, rows, off, idx = _grid_csr(grid)
    (w0, w1), (h0, h1) = window
    out = np.zeros(4096, np.int32)
    if lib is None:
        lib = load()
        n = lib.oracle_grid_candidates(cols, rows, _p(off), _p(idx), sp[0], sp[1], ep[0], ep[1], w0, w1, h0, h1,
                                       range_hint, _p(out), len(out))
    else:
        n = getattr(lib, fn)(cols, rows, _p(off), _p(idx), sp[0], sp[1], ep[0], ep[1], w0, w1, h0, h1, _p(out),
                             len(out))
    assert n <= len(out)
    return out[:n].tolist()


def line_coords(x1, y1, x2, y2, lib=None, fn="oracle_line_coords"):
    """getLineCoords (gridStructure.cpp:32-40) as (x, y) pairs."""
    lib = lib or load()
    out = np.zeros(2 * 8192, np.int32)
    n = getattr(lib, fn)(float(x1), float(y1), float(x2), float(y2), _p(out), 8192)
    assert n <= 8192
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def _declare_vocab(lib):
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.oracle_vocab_load.argtypes = [ctypes.c_char_p, I]
    lib.oracle_vocab_load.restype = V
    lib.oracle_vocab_create.argtypes = [I, I, I, I, I, V, V, V, V]
    lib.oracle_vocab_create.restype = V
    lib.oracle_vocab_free.argtypes = [V]
    lib.oracle_vocab_info.argtypes = [V, V]
    lib.oracle_vocab_nodes.argtypes = [V, V, V, V, V, V, V]
    lib.oracle_vocab_transform.argtypes = [V, V, I, I, V, V, V, V, V, V, V, V, V, V]


class Vocab:
    """DBoW2 TemplatedVocabulary restatement (oracle/bow_oracle.cpp)."""

    def __init__(self, handle):
        self.lib = load()
        _declare_vocab(self.lib)
        if not handle:
            raise ValueError("oracle vocabulary load failed")
        self.h = handle
        info = np.zeros(6, np.int32)
        self.lib.oracle_vocab_info(self.h, _p(info))
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = (int(x) for x in info)

    @classmethod
    def load_text(cls, path, emulate_tail=False):
        lib = load()
        _declare_vocab(lib)
        return cls(lib.oracle_vocab_load(str(path).encode(), int(emulate_tail)))

    @classmethod
    def create(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        lib = load()
        _declare_vocab(lib)
        parent = np.ascontiguousarray(parent, np.int32); is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8); weight = np.ascontiguousarray(weight, np.float64)
        h = lib.oracle_vocab_create(k, L, scoring, weighting, len(parent), _p(parent), _p(is_leaf), _p(desc),
                                    _p(weight))
        v = cls(h)
        v._keep = (parent, is_leaf, desc, weight)
        return v

    def __del__(self):
        try:
            self.lib.oracle_vocab_free(self.h)
        except Exception:
            pass

    def nodes(self):
        n = self.n_nodes
        parent, nchild = np.zeros(n, np.int32), np.zeros(n, np.int32)
        word, weight = np.zeros(n, np.uint32), np.zeros(n, np.float64)
        desc, children = np.zeros((n, 32), np.uint8), np.zeros(max(n, 1), np.int32)
        self.lib.oracle_vocab_nodes(self.h, _p(parent), _p(nchild), _p(word), _p(weight), _p(desc), _p(children))
        return parent, nchild, word, weight, desc

    def transform(self, desc, levelsup=4):
        """-> (bow_word, bow_value, fv_node, fv_off, fv_idx, feat_word, feat_w, feat_nid)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = d.shape[0]
        m = max(n, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fo, fi = np.zeros(m, np.uint32), np.zeros(m + 1, np.int32), np.zeros(m, np.uint32)
        fw, fwt, fni = np.zeros(m, np.uint32), np.zeros(m, np.float64), np.zeros(m, np.uint32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        self.lib.oracle_vocab_transform(self.h, _p(d), n, levelsup, _p(bw), _p(bv), ctypes.byref(nb), _p(fn), _p(fo),
                                        _p(fi), ctypes.byref(nf), _p(fw), _p(fwt), _p(fni))
        nb, nf = nb.value, nf.value
        return bw[:nb], bv[:nb], fn[:nf], fo[:nf + 1], fi[:fo[nf]], fw[:n], fwt[:n], fni[:n]


def assign_grid(kx, ky, grid):
    """Frame::AssignFeaturesToGrid restatement -> (cell_off[3073], cell_idx)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_assign_grid.argtypes = [V, V, I, F, F, F, F, V, V]
    lib.oracle_assign_grid.restype = I
    kx = np.ascontiguousarray(kx, np.float32); ky = np.ascontiguousarray(ky, np.float32)
    off = np.zeros(64 * 48 + 1, np.int32); idx = np.zeros(max(len(kx), 1), np.int32)
    min_x, max_x, min_y, max_y, inv_w, inv_h = grid
    m = lib.oracle_assign_grid(_p(kx), _p(ky), len(kx), min_x, min_y, inv_w, inv_h, _p(off), _p(idx))
    return off, idx[:m]


def features_in_area(kx, ky, oct_, grid, x, y, r, min_level, max_level):
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_features_in_area.argtypes = [V, V, V, I, F, F, F, F, F, F, F, I, I, V]
    lib.oracle_features_in_area.restype = I
    kx = np.ascontiguousarray(kx, np.float32); ky = np.ascontiguousarray(ky, np.float32)
    oc = np.ascontiguousarray(oct_, np.int32)
    out = np.zeros(max(len(kx), 1), np.int32)
    min_x, max_x, min_y, max_y, inv_w, inv_h = grid
    n = lib.oracle_features_in_area(_p(kx), _p(ky), _p(oc), len(kx), min_x, min_y, inv_w, inv_h, x, y, r,
                                    min_level, max_level, _p(out))
    return out[:n]


def search_by_projection(case, th, forward=0, backward=0, check_ori=1):
    """ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) restatement -> (nmatches, match)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_by_projection.argtypes = [I, V, V, V, V, V, V, V, F, F, F, F, F, F, V, F, F, F, F, F, I, V,
                                                V, V, V, V, F, I, I, I, V]
    lib.oracle_search_by_projection.restype = I
    c = case
    k = c["cur_kps"]
    kx = np.ascontiguousarray(k["x"], np.float32); ky = np.ascontiguousarray(k["y"], np.float32)
    ko = np.ascontiguousarray(k["octave"], np.int32); ka = np.ascontiguousarray(k["angle"], np.float32)
    cd = np.ascontiguousarray(c["cur_desc"], np.uint8)
    cb = np.ascontiguousarray(c["cur_blocked"], np.uint8)
    cu = None if c.get("cur_uright") is None else np.ascontiguousarray(c["cur_uright"], np.float32)
    min_x, max_x, min_y, max_y, inv_w, inv_h = c["grid"]
    sf = np.ascontiguousarray(c["scale_factors"], np.float32)
    x3 = np.ascontiguousarray(c["x3dc"], np.float32); lf = np.ascontiguousarray(c["flags"], np.uint8)
    lo = np.ascontiguousarray(c["last_octave"], np.int32); la = np.ascontiguousarray(c["last_angle"], np.float32)
    md = np.ascontiguousarray(c["mp_desc"], np.uint8)
    fx, fy, cx, cy, mbf = c["camera"]
    out = np.full(max(len(kx), 1), -1, np.int32)
    n = lib.oracle_search_by_projection(len(kx), _p(kx), _p(ky), _p(ko), _p(ka), _p(cd), _p(cb),
                                        None if cu is None else _p(cu), min_x, max_x, min_y, max_y, inv_w, inv_h,
                                        _p(sf), fx, fy, cx, cy, mbf, len(lf), _p(lf), _p(x3), _p(lo), _p(la), _p(md),
                                        th, forward, backward, check_ori, _p(out))
    return n, out[:len(kx)]


def search_by_projection_stereo(case, th, forward=0, backward=0, check_ori=1):
    """Two-camera SearchByProjection(CurrentFrame, LastFrame, th, bMono) restatement
    -> (nmatches, match_left, match_right)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_by_projection2.argtypes = [I, V, V, V, V, I, V, V, V, V, V, V, F, F, F, F, F, F, V, F, F, F,
                                                 F, V, I, V, V, V, V, V, V, F, I, I, I, V]
    lib.oracle_search_by_projection2.restype = I
    c = case
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    i32 = lambda a: np.ascontiguousarray(a, np.int32)  # noqa: E731
    kl, kr = c["kps"], c["kps_r"]
    nl, nr = len(kl), len(kr)
    lx, ly, lo, la = f32(kl["x"]), f32(kl["y"]), i32(kl["octave"]), f32(kl["angle"])
    rx, ry, ro, ra = f32(kr["x"]), f32(kr["y"]), i32(kr["octave"]), f32(kr["angle"])
    desc = np.ascontiguousarray(np.concatenate([c["desc"], c["desc_r"]]), np.uint8)
    blk = np.ascontiguousarray(np.concatenate([c["blocked"], c["blocked_r"]]), np.uint8)
    min_x, max_x, min_y, max_y, inv_w, inv_h = c["grid"]
    sf = f32(c["scale_factors"])
    fx, fy, cx, cy, _ = c["camera"]
    kb = None if c.get("kb8") is None else f32(c["kb8"])
    lf = np.ascontiguousarray(c["flags"], np.uint8)
    x3, x3r = f32(c["x3dc"]), f32(c["x3dr"])
    oc, an = i32(c["last_octave"]), f32(c["last_angle"])
    md = np.ascontiguousarray(c["mp_desc"], np.uint8)
    out = np.full(max(nl + nr, 1), -1, np.int32)
    n = lib.oracle_search_by_projection2(nl, _p(lx), _p(ly), _p(lo), _p(la), nr, _p(rx), _p(ry), _p(ro), _p(ra),
                                         _p(desc), _p(blk), min_x, max_x, min_y, max_y, inv_w, inv_h, _p(sf), fx, fy,
                                         cx, cy, None if kb is None else _p(kb), len(lf), _p(lf), _p(x3), _p(x3r),
                                         _p(oc), _p(an), _p(md), th, forward, backward, check_ori, _p(out))
    return n, out[:nl], out[nl:nl + nr]


def search_reloc(case, th, orb_dist, check_ori=1):
    """ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) restatement
    -> (nmatches, match)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_reloc.argtypes = [I, V, V, V, V, V, V, F, F, F, F, F, F, V, I, F, F, F, F, I, V, V, V, V, V,
                                        V, F, I, I, V]
    lib.oracle_search_reloc.restype = I
    c = case
    k = c["cur_kps"]
    kx = np.ascontiguousarray(k["x"], np.float32); ky = np.ascontiguousarray(k["y"], np.float32)
    ko = np.ascontiguousarray(k["octave"], np.int32); ka = np.ascontiguousarray(k["angle"], np.float32)
    cd = np.ascontiguousarray(c["cur_desc"], np.uint8)
    cb = np.ascontiguousarray(c["cur_blocked"], np.uint8)
    min_x, max_x, min_y, max_y, inv_w, inv_h = c["grid"]
    sf = np.ascontiguousarray(c["scale_factors"], np.float32)
    fl = np.ascontiguousarray(c["kf_flags"], np.uint8)
    x3 = np.ascontiguousarray(c["x3dc"], np.float32); ds = np.ascontiguousarray(c["dist"], np.float32)
    lv = np.ascontiguousarray(c["level"], np.int32); an = np.ascontiguousarray(c["kf_angle"], np.float32)
    md = np.ascontiguousarray(c["mp_desc"], np.uint8)
    fx, fy, cx, cy, _ = c["camera"]
    out = np.full(max(len(kx), 1), -1, np.int32)
    n = lib.oracle_search_reloc(len(kx), _p(kx), _p(ky), _p(ko), _p(ka), _p(cd), _p(cb), min_x, max_x, min_y, max_y,
                                inv_w, inv_h, _p(sf), len(sf), fx, fy, cx, cy, len(fl), _p(fl), _p(x3), _p(ds), _p(lv),
                                _p(an), _p(md), th, orb_dist, check_ori, _p(out))
    return n, out[:len(kx)]


def search_local(case, th, nnratio=0.8):
    """ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, ...) restatement -> (nmatches, match)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_local.argtypes = [I, V, V, V, V, V, V, F, F, F, F, V, F, F, I, V, V, V, V, V, V, V, V]
    lib.oracle_search_local.restype = I
    c = case
    k = c["cur_kps"]
    kx = np.ascontiguousarray(k["x"], np.float32); ky = np.ascontiguousarray(k["y"], np.float32)
    ko = np.ascontiguousarray(k["octave"], np.int32)
    cd = np.ascontiguousarray(c["cur_desc"], np.uint8)
    cb = np.ascontiguousarray(c["cur_blocked"], np.uint8)
    cu = None if c.get("cur_uright") is None else np.ascontiguousarray(c["cur_uright"], np.float32)
    min_x, _, min_y, _, inv_w, inv_h = c["grid"]
    sf = np.ascontiguousarray(c["scale_factors"], np.float32)
    fl = np.ascontiguousarray(c["mp_flags"], np.uint8)
    pr = np.ascontiguousarray(c["mp_proj"], np.float32)
    px, py, pxr, vc = (np.ascontiguousarray(pr[:, j]) for j in range(4))
    lv = np.ascontiguousarray(c["mp_level"], np.int32)
    md = np.ascontiguousarray(c["mp_desc"], np.uint8)
    out = np.full(max(len(kx), 1), -1, np.int32)
    n = lib.oracle_search_local(len(kx), _p(kx), _p(ky), _p(ko), _p(cd), _p(cb), None if cu is None else _p(cu),
                                min_x, min_y, inv_w, inv_h, _p(sf), nnratio, th, len(fl), _p(fl), _p(px), _p(py),
                                _p(pxr), _p(vc), _p(lv), _p(md), _p(out))
    return n, out[:len(kx)]


def search_local_stereo(case, th, nnratio=0.8):
    """Two-camera SearchByProjection(Frame&, const vector<MapPoint*>&, ...) restatement
    -> (nmatches, match_left, match_right)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_local2.argtypes = [I, V, V, V, I, V, V, V, V, V, V, V, F, F, F, F, V, F, F, I, V, V, V, V, V,
                                         V, V, V, V, V, V]
    lib.oracle_search_local2.restype = I
    c = case
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    i32 = lambda a: np.ascontiguousarray(a, np.int32)  # noqa: E731
    kl, kr = c["kps"], c["kps_r"]
    nl, nr = len(kl), len(kr)
    desc = np.ascontiguousarray(np.concatenate([c["desc"], c["desc_r"]]), np.uint8)
    blk = np.ascontiguousarray(np.concatenate([c["blocked"], c["blocked_r"]]), np.uint8)
    l2r, r2l = i32(c["l2r"]), i32(c["r2l"])
    min_x, _, min_y, _, inv_w, inv_h = c["grid"]
    sf = f32(c["scale_factors"])
    fl = np.ascontiguousarray(c["mp_flags"], np.uint8)
    pr, prr = f32(c["mp_proj"]), f32(c["mp_proj_r"])
    lv, lvr = i32(c["mp_level"]), i32(c["mp_level_r"])
    md = np.ascontiguousarray(c["mp_desc"], np.uint8)
    cols = [f32(pr[:, j]) for j in range(4)] + [f32(prr[:, j]) for j in range(4)]
    lx, ly, lo = f32(kl["x"]), f32(kl["y"]), i32(kl["octave"])
    rx, ry, ro = f32(kr["x"]), f32(kr["y"]), i32(kr["octave"])
    out = np.full(max(nl + nr, 1), -1, np.int32)
    n = lib.oracle_search_local2(nl, _p(lx), _p(ly), _p(lo), nr, _p(rx), _p(ry), _p(ro), _p(desc), _p(blk), _p(l2r),
                                 _p(r2l), min_x, min_y, inv_w, inv_h, _p(sf), nnratio, th, len(fl), _p(fl),
                                 _p(cols[0]), _p(cols[1]), _p(cols[3]), _p(lv), _p(cols[4]), _p(cols[5]), _p(cols[7]),
                                 _p(lvr), _p(md), _p(out))
    return n, out[:nl], out[nl:nl + nr]


def line_search_projection(case, th, angth, range_hint=1):
    """LineMatcher::SearchByProjection restatement -> (count, match)."""
    lib = load()
    V, I, F, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
    lib.oracle_line_search_projection.argtypes = [I, V, V, V, I, I, V, V, I, V, V, V, V, F, F, F, F, F, F, F, F, D, D,
                                                  V, F, F, I, V]
    lib.oracle_line_search_projection.restype = I
    c = case
    grid = c["grid"]
    cols, rows = len(grid), len(grid[0])
    off = np.zeros(cols * rows + 1, np.int32)
    flat = []
    for x in range(cols):
        for y in range(rows):
            flat.extend(grid[x][y])
            off[x * rows + y + 1] = len(flat)
    idx = np.array(flat if flat else [0], np.int32)
    ca = np.ascontiguousarray(c["cur_angle"], np.float32)
    cd = np.ascontiguousarray(c["cur_desc"], np.uint8)
    cb = np.ascontiguousarray(c["cur_blocked"], np.uint8)
    fl = np.ascontiguousarray(c["last_flags"], np.uint8)
    x3 = np.ascontiguousarray(c["x3dc"], np.float32)
    oc = np.ascontiguousarray(c["last_octave"], np.int32)
    md = np.ascontiguousarray(c["ml_desc"], np.uint8)
    sl = np.ascontiguousarray(c["scale_l"], np.float32)
    fx, fy, cx, cy = c["camera"]
    mnx, mxx, mny, mxy = c["bounds"]
    out = np.full(max(len(ca), 1), -1, np.int32)
    n = lib.oracle_line_search_projection(len(ca), _p(ca), _p(cd), _p(cb), cols, rows, _p(off), _p(idx), len(fl),
                                          _p(fl), _p(x3), _p(oc), _p(md), fx, fy, cx, cy, mnx, mxx, mny, mxy,
                                          c["inv_w"], c["inv_h"], _p(sl), th, angth, range_hint, _p(out))
    return n, out[:len(ca)]


def undistort_points(K4, dist, xy):
    lib = load()
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.oracle_undistort_points.argtypes = [V, V, I, V, I, V]
    K = np.ascontiguousarray(K4, np.float32); d = np.ascontiguousarray(dist, np.float32)
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    out = np.zeros_like(xy)
    lib.oracle_undistort_points(_p(K), _p(d), len(d), _p(xy), xy.shape[0], _p(out))
    return out


def image_bounds(K4, dist, cols, rows):
    lib = load()
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.oracle_image_bounds.argtypes = [V, V, I, I, I, V]
    K = np.ascontiguousarray(K4, np.float32); d = np.ascontiguousarray(dist, np.float32)
    b = np.zeros(4, np.float32)
    lib.oracle_image_bounds(_p(K), _p(d), len(d), cols, rows, _p(b))
    return b


def orb_pyramid(img, nfeatures=1000, scale=1.2, nlevels=8):
    """mvImagePyramid of the oracle extractor (list of uint8 levels)."""
    img = np.ascontiguousarray(img, np.uint8)
    out = []
    for level in range(nlevels):
        lvl = orb_stage(img, level, nfeatures, scale, nlevels)["pyr"]
        out.append(lvl)
    return out


def stereo_match(kpsL, descL, kpsR, descR, pyrL, pyrR, scale, inv_scale, mb, mbf):
    """Frame::ComputeStereoMatches restatement -> (nstereo, mvuRight, mvDepth)."""
    lib = load()
    V, F, I = ctypes.c_void_p, ctypes.c_float, ctypes.c_int
    lib.oracle_stereo_match.argtypes = [V, V, I, V, V, I, V, V, V, V, V, V, V, F, F, V, V]
    lib.oracle_stereo_match.restype = I
    kl = np.ascontiguousarray(kpsL).view(KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kpsR).view(KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(descL, np.uint8)
    dr = np.ascontiguousarray(descR, np.uint8)
    off = np.cumsum([0] + [lv.size for lv in pyrL[:-1]]).astype(np.int64)
    bl = np.concatenate([lv.ravel() for lv in pyrL])
    br = np.concatenate([lv.ravel() for lv in pyrR])
    w = np.array([lv.shape[1] for lv in pyrL], np.int32)
    h = np.array([lv.shape[0] for lv in pyrL], np.int32)
    sc = np.ascontiguousarray(scale, np.float32)
    inv = np.ascontiguousarray(inv_scale, np.float32)
    n = len(kl)
    ur = np.zeros(max(n, 1), np.float32)
    dp = np.zeros(max(n, 1), np.float32)
    k = lib.oracle_stereo_match(_p(kl), _p(dl), n, _p(kr), _p(dr), len(kr), _p(bl), _p(br), _p(off), _p(w), _p(h),
                                _p(sc), _p(inv), mb, mbf, _p(ur), _p(dp))
    return k, ur[:n], dp[:n]


def stereo_lines(klL, descL, klR, descR, klUn, width, height, mbf, range_hint=0):
    """Frame::ComputeStereoMatches_Lines restatement -> (nstereo, matches, disparity, depth, le)."""
    lib = load()
    V, F, I = ctypes.c_void_p, ctypes.c_float, ctypes.c_int
    lib.oracle_stereo_lines.argtypes = [V, V, I, V, V, I, V, I, I, F, I, V, V, V, V]
    lib.oracle_stereo_lines.restype = I

    def pts(k):
        k = np.ascontiguousarray(k).view(KEYLINE_DTYPE)
        return np.ascontiguousarray(np.stack([k["startPointX"], k["startPointY"], k["endPointX"], k["endPointY"]],
                                             1).astype(np.float32))
    a, b = pts(klL), pts(klR)
    u = a if klUn is None else pts(klUn)
    n = len(a)
    dl = np.ascontiguousarray(descL, np.uint8)
    dr = np.ascontiguousarray(descR, np.uint8)
    m = np.zeros(max(n, 1), np.int32)
    disp = np.zeros((max(n, 1), 2), np.float32)
    dep = np.zeros((max(n, 1), 2), np.float32)
    le = np.zeros((max(n, 1), 3), np.float64)
    k = lib.oracle_stereo_lines(_p(a), _p(dl), n, _p(b), _p(dr), len(b), _p(u), width, height, mbf, range_hint,
                                _p(m), _p(disp),
                                _p(dep), _p(le))
    return k, m[:n], disp[:n], dep[:n], le[:n]


def search_for_initialization(kps1, desc1, prev_xy, kps2, desc2, grid, window=100, nnratio=0.9, check_ori=True):
    """ORBmatcher::SearchForInitialization (oracle/proj_oracle.cpp).  kps in
    plvi.KEYPOINT_DTYPE (or any record with x, y, octave, angle); grid =
    (min_x, min_y, inv_w, inv_h).  Returns (nmatches, vnMatches12, vbPrevMatched)."""
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_search_for_initialization.argtypes = [I, V, V, V, V, V, V, I, V, V, V, V, V, F, F, F, F, I, F, I, V]
    lib.oracle_search_for_initialization.restype = I
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    i32 = lambda a: np.ascontiguousarray(a, np.int32)  # noqa: E731
    n1, n2 = len(kps1), len(kps2)
    x1, y1, o1, a1 = f32(kps1["x"]), f32(kps1["y"]), i32(kps1["octave"]), f32(kps1["angle"])
    x2, y2, o2, a2 = f32(kps2["x"]), f32(kps2["y"]), i32(kps2["octave"]), f32(kps2["angle"])
    d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
    d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
    pv = np.array(prev_xy, np.float32).reshape(-1, 2).copy()
    m = np.full(max(n1, 1), -1, np.int32)
    n = lib.oracle_search_for_initialization(n1, _p(x1), _p(y1), _p(o1), _p(a1), _p(d1), _p(pv), n2, _p(x2), _p(y2),
                                             _p(o2), _p(a2), _p(d2), *[float(g) for g in grid], int(window),
                                             float(nnratio), int(bool(check_ori)), _p(m))
    return n, m[:n1].copy(), pv


def line_search_init(d1, d2):
    """LineMatcher::SerachForInitialize + Frame::lineDescriptorMAD (oracle/match_oracle.cpp):
    returns (pairs n x 2 (query, train), (nn_mad, nn12_mad))."""
    lib = load()
    V, I = ctypes.c_void_p, ctypes.c_int
    lib.oracle_line_search_init.argtypes = [V, I, V, I, V, V, V]
    lib.oracle_line_search_init.restype = I
    d1 = np.ascontiguousarray(d1, np.uint8).reshape(-1, 32)
    d2 = np.ascontiguousarray(d2, np.uint8).reshape(-1, 32)
    q = np.zeros(max(len(d1), 1), np.int32)
    t = np.zeros(max(len(d1), 1), np.int32)
    mad = np.zeros(2, np.float64)
    n = lib.oracle_line_search_init(_p(d1), len(d1), _p(d2), len(d2), _p(q), _p(t), _p(mad))
    return np.stack([q[:n], t[:n]], 1), (float(mad[0]), float(mad[1]))


# ------------------------------------------------- frustum (oracle/frustum_oracle.cpp)
def _frustum_fns():
    lib = load()
    V, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    lib.oracle_predict_scale.argtypes = [F, F, F, I]
    lib.oracle_predict_scale.restype = I
    lib.oracle_level_table_check.argtypes = [V, F, I, F, F, ctypes.POINTER(ctypes.c_uint32)]
    lib.oracle_level_table_check.restype = ctypes.c_longlong
    lib.oracle_frustum_points.argtypes = [V, V, V, V, V, I, V, V, V, V, V, V]
    lib.oracle_frustum_points.restype = I
    lib.oracle_frustum_lines.argtypes = [V, V, V, V, V, I, V, V, V, V]
    lib.oracle_frustum_lines.restype = I
    lib.oracle_local_lines_filter.argtypes = [V, V, I, V, V, V, V, I, V, V]
    lib.oracle_local_lines_filter.restype = I
    return lib


def predict_scale(max_distance, dist, log_scale_factor, nlevels):
    """MapPoint::PredictScale (MapPoint.cc:531-546) with the host glibc logf."""
    return _frustum_fns().oracle_predict_scale(max_distance, dist, log_scale_factor, nlevels)


def level_table_check(thr, lsf, nlevels, lo, hi):
    """Mismatches of the threshold rule vs PredictScale over every float ratio in [lo, hi]."""
    t = np.ascontiguousarray(thr, np.float32)
    first = ctypes.c_uint32(0)
    bad = _frustum_fns().oracle_level_table_check(_p(t), float(lsf), int(nlevels), float(lo), float(hi),
                                                  ctypes.byref(first))
    return bad, first.value


def frustum_points(params, case):
    """Tracking.cc:5074-5092 over one frame (Frame::isInFrustum) -> dict of the MapPoint fields after it."""
    lib = _frustum_fns()
    n = len(case["pos"])
    pos = np.ascontiguousarray(case["pos"], np.float32)
    nr = np.ascontiguousarray(case["normal"], np.float32)
    ds = np.ascontiguousarray(case["dist"], np.float32)
    fi = np.ascontiguousarray(case["in_flags"], np.uint8)
    pr = np.array(case["proj"], np.float32)
    lv = np.array(case["level"], np.int32)
    de = np.array(case["depth"], np.float32)
    prr = np.array(case["proj_r"], np.float32)
    lvr = np.array(case["level_r"], np.int32)
    fo = np.zeros(max(n, 1), np.uint8)
    nv = lib.oracle_frustum_points(ctypes.byref(params), _p(pos), _p(nr), _p(ds), _p(fi), n, _p(fo), _p(pr), _p(lv),
                                   _p(prr), _p(lvr), _p(de))
    return {"nvisible": nv, "flags": fo[:n], "proj": pr, "level": lv, "depth": de, "proj_r": prr, "level_r": lvr}


def frustum_lines(params, case):
    """Tracking.cc:5219-5234 over one frame (Frame::isInFrustum_l) -> (inview, proj, angle, compact)."""
    lib = _frustum_fns()
    n = len(case["sep"])
    sp = np.ascontiguousarray(case["sep"], np.float64)
    nr = np.ascontiguousarray(case["normal"], np.float32)
    ds = np.ascontiguousarray(case["dist"], np.float32)
    fi = np.ascontiguousarray(case["in_flags"], np.uint8)
    pr = np.array(case["proj"], np.float32)
    an = np.array(case["angle"], np.float64)
    iv = np.zeros(max(n, 1), np.uint8)
    cp = np.zeros(max(n, 1), np.int32)
    nc = lib.oracle_frustum_lines(ctypes.byref(params), _p(sp), _p(nr), _p(ds), _p(fi), n, _p(iv), _p(pr), _p(an),
                                  _p(cp))
    return iv[:n], pr, an, cp[:nc].copy()


def local_lines_filter(params, matches_12, compact, proj, angle, keylines, blocked=None):
    """Tracking.cc:5244-5292 -> (nassigned, assign, matches_12 after)."""
    lib = _frustum_fns()
    m = np.array(matches_12, np.int32)
    cp = np.ascontiguousarray(compact, np.int32)
    pr = np.ascontiguousarray(proj, np.float32)
    an = np.ascontiguousarray(angle, np.float64)
    kl = np.ascontiguousarray(np.stack([keylines["startPointX"], keylines["startPointY"], keylines["endPointX"],
                                        keylines["endPointY"]], 1), np.float32)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    asg = np.full(max(len(kl), 1), -1, np.int32)
    na = lib.oracle_local_lines_filter(ctypes.byref(params), _p(m), len(cp), _p(cp), _p(pr), _p(an), _p(kl), len(kl),
                                       None if bl is None else _p(bl), _p(asg))
    return na, asg[:len(kl)], m
