"""Deterministic synthetic EuRoC-shaped frames.

numpy PCG64(seed); W×H u8.  Background = bilinear upsample of an 8×6 grid
U[60,190]; 40 filled rotated rectangles (intensity U[0,255]); 60 line
segments (width 1–3 px, contrast >= 40); Gaussian noise sigma=2, rint, clip.
The pair frame t+1 is frame t shifted by an integer (dx,dy) in [-3,3]^2
plus fresh noise.  Gives thousands of FAST corners at th=20 and >=200 LSD
segments per 640×480 frame.
"""
import numpy as np


def _background(rng, w, h):
    grid = rng.uniform(60, 190, size=(6, 8))
    ys = np.linspace(0, 5, h)
    xs = np.linspace(0, 7, w)
    y0 = np.clip(np.floor(ys).astype(int), 0, 4)
    x0 = np.clip(np.floor(xs).astype(int), 0, 6)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    return (g00 * (1 - fy) * (1 - fx) + g01 * (1 - fy) * fx + g10 * fy * (1 - fx) + g11 * fy * fx)


def _draw_rect(img, rng):
    h, w = img.shape
    cx, cy = rng.uniform(0, w), rng.uniform(0, h)
    a, b = rng.uniform(8, w / 6), rng.uniform(8, h / 6)
    th = rng.uniform(0, np.pi)
    val = rng.uniform(0, 255)
    r = int(np.ceil(np.hypot(a, b))) + 1
    x0, x1 = max(int(cx) - r, 0), min(int(cx) + r + 1, w)
    y0, y1 = max(int(cy) - r, 0), min(int(cy) + r + 1, h)
    if x0 >= x1 or y0 >= y1:
        return
    yy, xx = np.mgrid[y0:y1, x0:x1]
    dx, dy = xx - cx, yy - cy
    u = dx * np.cos(th) + dy * np.sin(th)
    v = -dx * np.sin(th) + dy * np.cos(th)
    m = (np.abs(u) <= a) & (np.abs(v) <= b)
    img[y0:y1, x0:x1][m] = val


def _draw_line(img, rng):
    h, w = img.shape
    x0, y0 = rng.uniform(0, w), rng.uniform(0, h)
    ang = rng.uniform(0, np.pi)
    ln = rng.uniform(30, 250)
    x1, y1 = x0 + ln * np.cos(ang), y0 + ln * np.sin(ang)
    width = rng.uniform(1, 3)
    bx0, bx1 = int(max(min(x0, x1) - 3, 0)), int(min(max(x0, x1) + 4, w))
    by0, by1 = int(max(min(y0, y1) - 3, 0)), int(min(max(y0, y1) + 4, h))
    if bx0 >= bx1 or by0 >= by1:
        return
    yy, xx = np.mgrid[by0:by1, bx0:bx1]
    px, py = xx - x0, yy - y0
    dx, dy = x1 - x0, y1 - y0
    t = np.clip((px * dx + py * dy) / (dx * dx + dy * dy), 0, 1)
    dist = np.hypot(px - t * dx, py - t * dy)
    m = dist <= width / 2
    region = img[by0:by1, bx0:bx1]
    base = float(np.median(region)) if region.size else 128.0
    c = rng.uniform(40, 120) * (1 if rng.uniform() < 0.5 else -1)
    val = np.clip(base + c, 0, 255)
    if abs(val - base) < 40:
        val = np.clip(base - c, 0, 255)
    region[m] = val


def clean_frame(seed, w=640, h=480):
    rng = np.random.Generator(np.random.PCG64(seed))
    img = _background(rng, w, h)
    for _ in range(40):
        _draw_rect(img, rng)
    for _ in range(60):
        _draw_line(img, rng)
    return img, rng


def _finish(img, rng):
    noisy = img + rng.normal(0.0, 2.0, size=img.shape)
    return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)


def frame(seed, w=640, h=480):
    """One synthetic frame (u8 H×W)."""
    img, rng = clean_frame(seed, w, h)
    return _finish(img, rng)


def frame_pair(seed, w=640, h=480):
    """(frame t, frame t+1): t+1 = integer shift of t's clean image + fresh noise."""
    img, rng = clean_frame(seed, w, h)
    dx, dy = rng.integers(-3, 4, size=2)
    shifted = np.roll(np.roll(img, int(dy), axis=0), int(dx), axis=1)
    a = _finish(img, rng)
    b = _finish(shifted, rng)
    return a, b


def stereo_pair(seed, w=640, h=480):
    """Rectified stereo pair (left, right, (d_top, d_bottom)): one clean image of width w + 64 seen by the
    left camera at columns [0, w) and by the right camera shifted by an integer disparity, d_top for the upper
    half of the rows and d_bottom for the lower half (two depth planes), each side with its own noise."""
    img, rng = clean_frame(seed, w + 64, h)
    d0, d1 = (int(v) for v in rng.integers(4, 60, size=2))
    left = img[:, :w]
    right = np.empty((h, w))
    right[: h // 2] = img[: h // 2, d0:d0 + w]
    right[h // 2:] = img[h // 2:, d1:d1 + w]
    return _finish(left, rng), _finish(right, rng), (d0, d1)


def batch(n, w=640, h=480, seed0=0):
    """n frames with seeds seed0..seed0+n-1 as one contiguous (n,H,W) u8 array."""
    out = np.empty((n, h, w), np.uint8)
    for i in range(n):
        out[i] = frame(seed0 + i, w, h)
    return out


def device_sequence(n, w=640, h=480, seed=0, device="cpu", run=48):
    """n consecutive frames of a synthetic camera sequence, generated on
    `device` (torch) into one contiguous (n, H, W) u8 tensor -- the bench's
    input, so that thousands of frames per GPU need no host generation.

    Runs of `run` frames share one clean scene (clean_frame(seed + k*run),
    the numpy generator above); within a run frame t+1 is frame t shifted by
    an integer (dx, dy) in [-3, 3]^2 (seeded, cumulative, np.roll wrap) plus
    fresh Gaussian noise sigma 2 (torch generator seeded with `seed`),
    round-half-even and clip to [0, 255] -- SURVEY 8(d)'s pair rule applied
    along a sequence.  Deterministic for a given (n, w, h, seed, device type)."""
    import torch
    out = torch.empty((n, h, w), dtype=torch.uint8, device=device)
    if n == 0:
        return out
    steps = np.random.default_rng(seed ^ 0x5EED5EED).integers(-3, 4, size=(n, 2))
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
    for k in range((n + run - 1) // run):
        lo, hi = k * run, min(n, (k + 1) * run)
        base = torch.from_numpy(clean_frame(seed + lo, w, h)[0]).to(device=device, dtype=torch.float32)
        sh = np.cumsum(steps[lo:hi], axis=0)
        sh -= sh[0]
        noise = torch.randn((hi - lo, h, w), generator=g, device=device) * 2.0
        for t in range(lo, hi):
            img = torch.roll(base, shifts=(int(sh[t - lo, 1]), int(sh[t - lo, 0])), dims=(0, 1))
            out[t] = torch.clamp(torch.round(img + noise[t - lo]), 0, 255).to(torch.uint8)
    return out


# ---------------------------------------------------------------- vocabulary
# Seeded synthetic DBoW2 ORB vocabulary in the reference's node-table form
# (the real Vocabulary/ORBvoc.txt is a missing blob).
# Children of a node are consecutive in file order, as the kmeans builder
# creates them; descriptors of a child = its parent's with random bit flips,
# so descending the tree is meaningful; leaves carry idf-like weights with
# ~2 % stopped words (weight 0).

def _flip_mask(rng, n, ands):
    """n x 32 random bytes whose bits are set with probability 2^-ands."""
    m = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    for _ in range(ands - 1):
        m &= rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return m


def vocabulary(k=10, L=6, seed=0):
    """Full k-ary tree of depth L in breadth-first file order.
    Returns (parent, is_leaf, desc, weight) for nodes 1..n."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parents, leaves, descs, weights = [], [], [], []
    prev_ids = np.zeros(1, np.int64)
    prev_desc = np.zeros((1, 32), np.uint8)
    next_id = 1
    for d in range(1, L + 1):
        cnt = len(prev_ids) * k
        par = np.repeat(prev_ids, k)
        if d == 1:
            de = rng.integers(0, 256, (cnt, 32), dtype=np.uint8)
        else:
            de = np.repeat(prev_desc, k, axis=0) ^ _flip_mask(rng, cnt, min(d, 5))
        ids = np.arange(next_id, next_id + cnt, dtype=np.int64)
        next_id += cnt
        leaf = d == L
        w = np.zeros(cnt)
        if leaf:
            w = rng.uniform(0.5, 9.0, cnt)
            w[rng.uniform(size=cnt) < 0.02] = 0.0
        parents.append(par)
        leaves.append(np.full(cnt, leaf, np.uint8))
        descs.append(de)
        weights.append(w)
        prev_ids, prev_desc = ids, de
    return (np.concatenate(parents).astype(np.int32), np.concatenate(leaves), np.concatenate(descs),
            np.concatenate(weights))


def vocabulary_irregular(k=6, L=4, seed=0):
    """Small irregular tree in the kmeans builder's file order (children of a
    node consecutive, recursion depth first): branching 1..k, early leaves,
    duplicate child descriptors (ties), stopped words."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, leaf, desc, weight = [], [], [], []

    def emit(pid, d, pdesc):
        nc = int(rng.integers(1, k + 1))
        first = len(parent) + 1
        kids = []
        for c in range(nc):
            if d == 1:
                de = rng.integers(0, 256, 32, dtype=np.uint8)
            elif c > 0 and rng.uniform() < 0.1:
                de = desc[kids[-1] - 1].copy()  # exact tie with the previous sibling
            else:
                de = pdesc ^ _flip_mask(rng, 1, 3)[0]
            is_leaf = d == L or (d >= 2 and rng.uniform() < 0.15)
            parent.append(pid)
            leaf.append(1 if is_leaf else 0)
            desc.append(de)
            weight.append(0.0 if (not is_leaf or rng.uniform() < 0.05) else float(rng.uniform(0.1, 5.0)))
            kids.append(first + c)
        for c, nid in enumerate(kids):
            if not leaf[nid - 1]:
                emit(nid, d + 1, desc[nid - 1])

    emit(0, 1, None)
    return (np.array(parent, np.int32), np.array(leaf, np.uint8), np.array(desc, np.uint8).reshape(-1, 32),
            np.array(weight, np.float64))


def vocabulary_text(k, L, scoring, weighting, parent, is_leaf, desc, weight):
    """saveToTextFile (TemplatedVocabulary.h:1429-1449) formatting."""
    lines = [f"{k} {L}  {scoring} {weighting}"]
    for p, lf, d, w in zip(parent, is_leaf, desc, weight):
        lines.append(f"{int(p)} {int(lf)} " + " ".join(str(int(x)) for x in d) + f"  {w:.6g}")
    return "\n".join(lines) + "\n"


def vocab_features(parent, is_leaf, desc, n, seed=0, flips=3):
    """n query descriptors near random leaves (bit flips with probability 2^-flips)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    leaves = np.nonzero(is_leaf)[0]
    pick = rng.choice(leaves, n)
    return desc[pick] ^ _flip_mask(rng, n, flips)
