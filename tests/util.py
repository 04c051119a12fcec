import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def real_frames():
    z = np.load(GOLDEN / "frames.npz")
    return {k: z[k] for k in z.files}


def near_duplicate_descriptors(rng, n_train, n_query, frac=0.6, p_flip=0.08):
    """C3 generator: 60% of queries are train rows with
    Binomial(256, p) bit flips, the rest uniform random bits."""
    t = rng.integers(0, 256, size=(n_train, 32), dtype=np.uint8)
    q = rng.integers(0, 256, size=(n_query, 32), dtype=np.uint8)
    k = int(frac * n_query)
    src = rng.integers(0, n_train, size=k)
    bits = np.unpackbits(t[src], axis=1)
    flips = rng.random(bits.shape) < p_flip
    q[:k] = np.packbits(bits ^ flips, axis=1)
    return q, t


def bow_case(seed, n_kf=1000, n_f=1000, n_nodes=100, zipf=1.2, live=0.7, dup=0.6, flips=0.08, rot=20.0):
    """Synthetic SearchByBoW input: NodeIds from a Zipf
    over n_nodes, 70 % live MapPoints, dup of the F rows are KF rows with
    Binomial(256, flips) bit flips in the same node, angles rotated by `rot`
    degrees plus noise.  Returns (kf_desc, kf_angle, kf_live, kf_fv, f_desc,
    f_angle, f_fv) with fv = {node: [indices ascending]}."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n_nodes + 1) ** zipf
    w /= w.sum()
    node_ids = np.sort(rng.choice(100000, n_nodes, replace=False))
    kf_desc = rng.integers(0, 256, (n_kf, 32), dtype=np.uint8)
    kf_node = node_ids[rng.choice(n_nodes, n_kf, p=w)]
    kf_angle = rng.uniform(0, 360, n_kf).astype(np.float32)
    kf_live = (rng.random(n_kf) < live).astype(np.uint8)
    f_desc = rng.integers(0, 256, (n_f, 32), dtype=np.uint8)
    f_node = node_ids[rng.choice(n_nodes, n_f, p=w)]
    f_angle = rng.uniform(0, 360, n_f).astype(np.float32)
    nd = int(dup * n_f)
    src = rng.choice(n_kf, nd, replace=True)
    bits = np.unpackbits(kf_desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < flips).astype(np.uint8)
    f_desc[:nd] = np.packbits(bits, axis=1)
    f_node[:nd] = kf_node[src]
    f_angle[:nd] = np.mod(kf_angle[src] - rot + rng.normal(0, 3, nd), 360).astype(np.float32)
    perm = rng.permutation(n_f)
    f_desc, f_node, f_angle = f_desc[perm], f_node[perm], f_angle[perm]

    def fv(nodes):
        d = {}
        for i, n in enumerate(nodes):
            d.setdefault(int(n), []).append(i)
        return d
    return kf_desc, kf_angle, kf_live, fv(kf_node), f_desc, f_angle, fv(f_node)


def line_iterator(x1, y1, x2, y2):
    """ORB_SLAM3::LineIterator (src/LineIterator.cpp:31-73): Bresenham on doubles."""
    steep = abs(y2 - y1) > abs(x2 - x1)
    if steep:
        x1, y1, x2, y2 = y1, x1, y2, x2
    if x1 > x2:
        x1, x2, y1, y2 = x2, x1, y2, y1
    dx, dy = x2 - x1, abs(y2 - y1)
    error = dx / 2.0
    ystep = 1 if y1 < y2 else -1
    x, y, maxX = int(x1), int(y1), int(x2)
    out = []
    while x <= maxX:
        out.append((y, x) if steep else (x, y))
        error -= dy
        if error < 0:
            y += ystep
            error += dx
        x += 1
    return out


def stereo_line_case(seed, n=220, W=640, H=480, cols=64, rows=48, ties=True):
    """Synthetic stereo line set shaped like Frame::ComputeStereoMatches_Lines
    (src/Frame.cc:1408-1451): right lines rasterised into the 64x48 grid with
    LineIterator, normalised directions, left lines = right lines shifted by a
    disparity with noisy descriptors.  Returns (lines1 int n1x4, desc1, grid,
    desc2, directions2)."""
    rng = np.random.default_rng(seed)
    inv_w, inv_h = cols / W, rows / H
    sp = np.stack([rng.uniform(0, W - 1, n), rng.uniform(0, H - 1, n)], 1)
    ang = rng.uniform(0, np.pi, n)
    ln = rng.uniform(5, 160, n)
    ep = np.clip(sp + np.stack([np.cos(ang), np.sin(ang)], 1) * ln[:, None], 0, [W - 1, H - 1])
    desc2 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if ties:  # duplicated right lines/descriptors produce distance ties
        k = n // 10
        desc2[-k:] = desc2[:k]
        sp[-k:] = sp[:k] + rng.normal(0, 2, (k, 2))
        ep[-k:] = ep[:k] + rng.normal(0, 2, (k, 2))
    grid = [[[] for _ in range(rows)] for _ in range(cols)]
    dirs = np.zeros((n, 2))
    for i in range(n):
        v = ((ep[i, 0] - sp[i, 0]) * inv_w, (ep[i, 1] - sp[i, 1]) * inv_h)
        m = np.sqrt(v[0] * v[0] + v[1] * v[1])
        dirs[i] = (v[0] / m, v[1] / m)
        for (x, y) in line_iterator(sp[i, 0] * inv_w, sp[i, 1] * inv_h, ep[i, 0] * inv_w, ep[i, 1] * inv_h):
            if 0 <= x < cols and 0 <= y < rows:
                grid[x][y].append(i)
    n1 = int(n * 0.9)
    src = rng.permutation(n)[:n1]
    disp = rng.uniform(2, 40, n1)
    s1 = sp[src] + np.stack([disp, np.zeros(n1)], 1)
    e1 = ep[src] + np.stack([disp, np.zeros(n1)], 1)
    bits = np.unpackbits(desc2[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.1).astype(np.uint8)
    desc1 = np.packbits(bits, axis=1)
    lines1 = np.stack([(s1[:, 0] * inv_w).astype(np.int64), (s1[:, 1] * inv_h).astype(np.int64),
                       (e1[:, 0] * inv_w).astype(np.int64), (e1[:, 1] * inv_h).astype(np.int64)], 1).astype(np.int32)
    return lines1, desc1, grid, desc2, dirs


def orb_scale_factors(n=8, sf=1.2):
    """ORBextractor mvScaleFactor (float cumulative, ORBextractor.cc:415-420)."""
    s = [np.float32(1.0)]
    for _ in range(1, n):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(sf))))
    return np.array(s + [np.float32(0)] * (16 - n), np.float32)


def projection_case(seed, n_cur=1000, n_last=900, W=752, H=480, uright=False, dup=0.05):
    """Synthetic SearchByProjection input: current-frame
    keypoints (mvKeysUn) with descriptors; LastFrame MapPoints whose camera-
    frame positions project near a current keypoint (70 %) or anywhere (30 %),
    descriptors = the keypoint's with ~5 % bit flips (or random), a global
    rotation of 10 degrees; some points invalid / behind the camera / with
    Observations() == 0, some current keypoints pre-blocked, `dup` of the
    last points aimed at the same keypoint as another (assignment conflicts)."""
    from plvi import KEYPOINT_DTYPE, grid_geometry
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = np.float32(458.654), np.float32(457.296), np.float32(367.215), np.float32(248.375)
    kps = np.zeros(n_cur, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(-4, W + 4, n_cur).astype(np.float32)
    kps["y"] = rng.uniform(-4, H + 4, n_cur).astype(np.float32)
    kps["octave"] = np.minimum(rng.geometric(0.35, n_cur) - 1, 7)
    kps["angle"] = rng.uniform(0, 360, n_cur).astype(np.float32)
    kps["size"] = 31
    kps["class_id"] = -1
    desc = rng.integers(0, 256, (n_cur, 32), dtype=np.uint8)
    near = rng.random(n_last) < 0.7
    src = rng.integers(0, n_cur, n_last)
    ndup = int(dup * n_last)
    src[:ndup] = src[ndup:2 * ndup]
    u = np.where(near, kps["x"][src] + rng.normal(0, 2.0, n_last), rng.uniform(0, W, n_last))
    v = np.where(near, kps["y"][src] + rng.normal(0, 2.0, n_last), rng.uniform(0, H, n_last))
    z = rng.uniform(1.0, 20.0, n_last)
    z[rng.random(n_last) < 0.02] *= -1
    x3 = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1).astype(np.float32)
    oct_ = np.clip(np.where(near, kps["octave"][src] + rng.integers(-1, 2, n_last), rng.integers(0, 8, n_last)), 0, 7)
    bits = np.unpackbits(desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.05).astype(np.uint8)
    mp = np.where(near[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (n_last, 32), dtype=np.uint8))
    ang = np.mod(kps["angle"][src] + 10 + rng.normal(0, 5, n_last), 360).astype(np.float32)
    flags = ((rng.random(n_last) < 0.92).astype(np.uint8) | ((rng.random(n_last) < 0.85).astype(np.uint8) << 1))
    case = {"cur_kps": kps, "cur_desc": desc, "cur_blocked": (rng.random(n_cur) < 0.05).astype(np.uint8),
            "cur_uright": None, "grid": grid_geometry(W, H), "scale_factors": orb_scale_factors(),
            "x3dc": x3, "flags": flags, "last_octave": oct_.astype(np.int32), "last_angle": ang,
            "mp_desc": mp.astype(np.uint8), "camera": (fx, fy, cx, cy, np.float32(40.0))}
    if uright:
        ur = np.where(rng.random(n_cur) < 0.6, kps["x"] - rng.uniform(0, 30, n_cur), -1).astype(np.float32)
        case["cur_uright"] = ur
    return case


KB8_TUMVI = (np.float32(190.978), np.float32(190.973), np.float32(254.932), np.float32(256.897),
             np.float32(0.0034823894), np.float32(0.00071503044), np.float32(-0.0020532361), np.float32(0.00020293143))


def _kb8_unproject(u, v, cam):
    """Rays (x/z, y/z) of pixels under KannalaBrandt8 (Newton on r(theta) = theta_d, float64)."""
    fx, fy, cx, cy, k1, k2, k3, k4 = (float(t) for t in cam)
    px, py = (u - cx) / fx, (v - cy) / fy
    td = np.minimum(np.hypot(px, py), np.pi / 2 - 1e-3)
    th = td.copy()
    for _ in range(20):
        t2 = th * th
        f = th * (1 + k1 * t2 + k2 * t2 ** 2 + k3 * t2 ** 3 + k4 * t2 ** 4) - td
        fd = 1 + 3 * k1 * t2 + 5 * k2 * t2 ** 2 + 7 * k3 * t2 ** 3 + 9 * k4 * t2 ** 4
        th = th - f / fd
    sc = np.where(td > 1e-8, np.tan(th) / np.maximum(td, 1e-12), 1.0)
    return px * sc, py * sc


def _kb8_project(x3, cam):
    fx, fy, cx, cy, k1, k2, k3, k4 = (float(t) for t in cam)
    x, y, z = x3[:, 0].astype(np.float64), x3[:, 1].astype(np.float64), x3[:, 2].astype(np.float64)
    th = np.arctan2(np.hypot(x, y), z)
    psi = np.arctan2(y, x)
    r = th + k1 * th ** 3 + k2 * th ** 5 + k3 * th ** 7 + k4 * th ** 9
    return fx * r * np.cos(psi) + cx, fy * r * np.sin(psi) + cy


def projection_stereo_case(seed, n_left=900, n_right=850, n_last=800, kb8=True, dup=0.05):
    """Two-camera SearchByProjection(CurrentFrame, LastFrame) input (CurrentFrame.Nleft != -1): a
    KannalaBrandt8 rig (TUM-VI-like intrinsics, 512 x 512, or a Pinhole one), left / right keypoints with
    descriptors, LastFrame points whose x3Dc project near a left keypoint (70 %) and whose x3Dr = Rrl x3Dc +
    trl project near a right keypoint placed there for 60 % of them (descriptor = the same source with flipped
    bits), a global 10-degree rotation, some points behind the camera / outliers / with Observations() == 0,
    pre-blocked keypoints on both sides, `dup` aimed at another point's keypoints."""
    from plvi import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    W = H = 512
    cam = KB8_TUMVI if kb8 else (np.float32(190.978), np.float32(190.973), np.float32(254.932),
                                 np.float32(256.897))

    def kset(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(-4, W + 4, n).astype(np.float32)
        k["y"] = rng.uniform(-4, H + 4, n).astype(np.float32)
        k["octave"] = np.minimum(rng.geometric(0.35, n) - 1, 7)
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        k["size"] = 31
        k["class_id"] = -1
        return k
    kl, kr = kset(n_left), kset(n_right)
    dl = rng.integers(0, 256, (n_left, 32), dtype=np.uint8)
    dr = rng.integers(0, 256, (n_right, 32), dtype=np.uint8)
    near = rng.random(n_last) < 0.7
    src = rng.integers(0, n_left, n_last)
    nd = int(dup * n_last)
    src[:nd] = src[nd:2 * nd]
    u = np.where(near, kl["x"][src] + rng.normal(0, 2.0, n_last), rng.uniform(0, W, n_last))
    v = np.where(near, kl["y"][src] + rng.normal(0, 2.0, n_last), rng.uniform(0, H, n_last))
    z = rng.uniform(1.0, 20.0, n_last)
    if kb8:
        rx_, ry_ = _kb8_unproject(u, v, cam)
    else:
        rx_, ry_ = (u - float(cam[2])) / float(cam[0]), (v - float(cam[3])) / float(cam[1])
    x3 = np.stack([rx_ * z, ry_ * z, z], 1)
    x3[rng.random(n_last) < 0.02] *= -1
    x3 = x3.astype(np.float32)
    a = np.deg2rad(2.0)
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    x3r = (x3.astype(np.float64) @ R.T + np.array([-0.11, 0.002, 0.001])).astype(np.float32)
    if kb8:
        ur, vr = _kb8_project(x3r, cam)
    else:
        ur = float(cam[0]) * x3r[:, 0] / x3r[:, 2] + float(cam[2])
        vr = float(cam[1]) * x3r[:, 1] / x3r[:, 2] + float(cam[3])
    # right keypoints at the right projections of 60 % of the near points
    put = np.nonzero(near & (rng.random(n_last) < 0.6) & (x3[:, 2] > 0))[0][:n_right]
    slots = rng.choice(n_right, len(put), replace=False)
    kr["x"][slots] = (ur[put] + rng.normal(0, 1.5, len(put))).astype(np.float32)
    kr["y"][slots] = (vr[put] + rng.normal(0, 1.5, len(put))).astype(np.float32)
    kr["octave"][slots] = kl["octave"][src[put]]
    kr["angle"][slots] = np.mod(kl["angle"][src[put]] + rng.normal(0, 3, len(put)), 360).astype(np.float32)
    bits = np.unpackbits(dl[src[put]], axis=1)
    bits ^= (rng.random(bits.shape) < 0.04).astype(np.uint8)
    dr[slots] = np.packbits(bits, axis=1)
    oct_ = np.clip(np.where(near, kl["octave"][src] + rng.integers(-1, 2, n_last), rng.integers(0, 8, n_last)), 0, 7)
    bits = np.unpackbits(dl[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.05).astype(np.uint8)
    mp = np.where(near[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (n_last, 32), dtype=np.uint8))
    ang = np.mod(kl["angle"][src] + 10 + rng.normal(0, 5, n_last), 360).astype(np.float32)
    flags = ((rng.random(n_last) < 0.92).astype(np.uint8) | ((rng.random(n_last) < 0.85).astype(np.uint8) << 1))
    cols, rows = 64, 48
    grid = (np.float32(0), np.float32(W), np.float32(0), np.float32(H), np.float32(cols / W), np.float32(rows / H))
    return {"kps": kl, "desc": dl, "kps_r": kr, "desc_r": dr,
            "blocked": (rng.random(n_left) < 0.05).astype(np.uint8),
            "blocked_r": (rng.random(n_right) < 0.05).astype(np.uint8), "grid": grid,
            "scale_factors": orb_scale_factors(), "x3dc": x3, "x3dr": x3r, "flags": flags,
            "last_octave": oct_.astype(np.int32), "last_angle": ang, "mp_desc": mp.astype(np.uint8),
            "camera": tuple(cam[:4]) + (np.float32(0.0),), "kb8": np.array(cam[4:], np.float32) if kb8 else None}


def reloc_case(seed, n_cur=1000, n_kf=800, W=752, H=480, dup=0.08, pre_blocked=0.3):
    """Synthetic relocalization-search input (ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound,
    th, ORBdist), src/ORBmatcher.cc:2180-2300): current-frame keypoints (mvKeysUn) with descriptors, ~30 %
    already holding a MapPoint (the PnP inliers); KF MapPoints that project near a keypoint (70 %) or anywhere,
    descriptors = the keypoint's with ~6 % bit flips (or random), dist3D inside / outside the MapPoints'
    distance invariance range, PredictScale levels = the keypoint's octave +-1 (a few at the clamp ends), some
    points dead or already found, `dup` aimed at another point's keypoint (assignment conflicts), a global
    rotation of 10 degrees plus noise, points behind the camera (the reloc search has no depth test)."""
    from plvi import KEYPOINT_DTYPE, grid_geometry
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = np.float32(458.654), np.float32(457.296), np.float32(367.215), np.float32(248.375)
    kps = np.zeros(n_cur, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(-4, W + 4, n_cur).astype(np.float32)
    kps["y"] = rng.uniform(-4, H + 4, n_cur).astype(np.float32)
    kps["octave"] = np.minimum(rng.geometric(0.35, n_cur) - 1, 7)
    kps["angle"] = rng.uniform(0, 360, n_cur).astype(np.float32)
    kps["size"] = 31
    kps["class_id"] = -1
    desc = rng.integers(0, 256, (n_cur, 32), dtype=np.uint8)
    near = rng.random(n_kf) < 0.7
    src = rng.integers(0, n_cur, n_kf)
    ndup = int(dup * n_kf)
    src[:ndup] = src[ndup:2 * ndup]
    u = np.where(near, kps["x"][src] + rng.normal(0, 2.0, n_kf), rng.uniform(-20, W + 20, n_kf))
    v = np.where(near, kps["y"][src] + rng.normal(0, 2.0, n_kf), rng.uniform(-20, H + 20, n_kf))
    z = rng.uniform(1.0, 20.0, n_kf)
    z[rng.random(n_kf) < 0.02] *= -1
    x3 = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1).astype(np.float32)
    d3 = np.abs(z * rng.uniform(1.0, 1.3, n_kf)).astype(np.float32)
    lo = (d3 * rng.uniform(0.3, 1.02, n_kf)).astype(np.float32)
    hi = (d3 * rng.uniform(0.98, 3.0, n_kf)).astype(np.float32)
    dist = np.stack([d3, lo, hi], 1).astype(np.float32)
    lvl = np.clip(np.where(near, kps["octave"][src] + rng.integers(-1, 2, n_kf), rng.integers(0, 8, n_kf)), 0, 7)
    bits = np.unpackbits(desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.06).astype(np.uint8)
    mp = np.where(near[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (n_kf, 32), dtype=np.uint8))
    ang = np.mod(kps["angle"][src] + 10 + rng.normal(0, 5, n_kf), 360).astype(np.float32)
    return {"cur_kps": kps, "cur_desc": desc, "cur_blocked": (rng.random(n_cur) < pre_blocked).astype(np.uint8),
            "grid": grid_geometry(W, H), "scale_factors": orb_scale_factors(), "x3dc": x3, "dist": dist,
            "level": lvl.astype(np.int32), "kf_flags": (rng.random(n_kf) < 0.9).astype(np.uint8),
            "kf_angle": ang, "mp_desc": mp.astype(np.uint8), "camera": (fx, fy, cx, cy, np.float32(0.0))}


def reloc_params(case, th, orb_dist):
    import plvi
    p = plvi.RelocParams()
    fx, fy, cx, cy, _ = case["camera"]
    p.fx, p.fy, p.cx, p.cy, p.th, p.orb_dist = fx, fy, cx, cy, th, orb_dist
    (p.min_x, p.max_x, p.min_y, p.max_y, p.inv_w, p.inv_h) = case["grid"]
    p.nlevels = len(case["scale_factors"])
    for i, s in enumerate(case["scale_factors"]):
        p.scale_factors[i] = s
    return p


def local_case(seed, n_cur=1000, n_mp=1500, W=752, H=480, uright=False, dup=0.15):
    """Synthetic local-map search input (ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>...),
    SURVEY 8f / VERDICT r1 item 8): current-frame keypoints with octaves and descriptors; MapPoints whose
    predicted projections fall near a keypoint (75 %) or anywhere, predicted level = the keypoint's octave
    +-1, descriptors = the keypoint's with ~6 % bit flips (ties and near-ties via duplicated MapPoints:
    `dup` of them aim at an earlier MapPoint's keypoint, so the sequential blocking matters), some not in
    view / bad, most with Observations() > 0, a few keypoints pre-blocked; view cosines on both sides of
    RadiusByViewingCos's 0.998."""
    from plvi import KEYPOINT_DTYPE, grid_geometry
    rng = np.random.default_rng(seed)
    kps = np.zeros(n_cur, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(-3, W + 3, n_cur).astype(np.float32)
    kps["y"] = rng.uniform(-3, H + 3, n_cur).astype(np.float32)
    kps["octave"] = np.minimum(rng.geometric(0.35, n_cur) - 1, 7)
    kps["size"] = 31
    kps["class_id"] = -1
    desc = rng.integers(0, 256, (n_cur, 32), dtype=np.uint8)
    near = rng.random(n_mp) < 0.75
    src = rng.integers(0, n_cur, n_mp)
    nd = int(dup * n_mp)
    if nd:
        src[-nd:] = src[rng.integers(0, n_mp - nd, nd)]
    px = np.where(near, kps["x"][src] + rng.normal(0, 1.5, n_mp), rng.uniform(0, W, n_mp)).astype(np.float32)
    py = np.where(near, kps["y"][src] + rng.normal(0, 1.5, n_mp), rng.uniform(0, H, n_mp)).astype(np.float32)
    pxr = (px - rng.uniform(0, 30, n_mp)).astype(np.float32)
    vc = np.where(rng.random(n_mp) < 0.5, rng.uniform(0.999, 1.0, n_mp), rng.uniform(0.5, 0.998, n_mp)).astype(
        np.float32)
    lvl = np.clip(np.where(near, kps["octave"][src] + rng.integers(-1, 2, n_mp), rng.integers(0, 8, n_mp)), 0, 7)
    bits = np.unpackbits(desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.06).astype(np.uint8)
    md = np.where(near[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (n_mp, 32), dtype=np.uint8))
    flags = ((rng.random(n_mp) < 0.9).astype(np.uint8) | ((rng.random(n_mp) < 0.85).astype(np.uint8) << 1))
    case = {"cur_kps": kps, "cur_desc": desc, "cur_blocked": (rng.random(n_cur) < 0.05).astype(np.uint8),
            "cur_uright": None, "grid": grid_geometry(W, H), "scale_factors": orb_scale_factors(),
            "mp_flags": flags, "mp_proj": np.stack([px, py, pxr, vc], 1).astype(np.float32),
            "mp_level": lvl.astype(np.int32), "mp_desc": md.astype(np.uint8)}
    if uright:
        case["cur_uright"] = np.where(rng.random(n_cur) < 0.6, kps["x"] - rng.uniform(0, 30, n_cur), -1).astype(
            np.float32)
    return case


def local_stereo_case(seed, n_left=900, n_right=850, n_mp=1400, W=752, H=480, pair_frac=0.6, dup=0.15):
    """Two-camera local-map search input (F.Nleft != -1): left / right keypoint sets with descriptors, a
    fraction of them paired (mvLeftToRightMatch / mvRightToLeftMatch, mutually consistent, right
    descriptor = the left one with a few flipped bits); MapPoints seen in the left image, the right image or
    both (bit0 / bit2), each aiming near a keypoint of that image (its predicted level = the keypoint's
    octave +-1, the right level sometimes -1), duplicates aiming at an earlier MapPoint's keypoints so the
    sequential blocking and the stereo cross-assignments matter."""
    from plvi import KEYPOINT_DTYPE, grid_geometry
    rng = np.random.default_rng(seed)

    def kset(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(-3, W + 3, n).astype(np.float32)
        k["y"] = rng.uniform(-3, H + 3, n).astype(np.float32)
        k["octave"] = np.minimum(rng.geometric(0.35, n) - 1, 7)
        k["size"] = 31
        k["class_id"] = -1
        return k
    kl, kr = kset(n_left), kset(n_right)
    dl = rng.integers(0, 256, (n_left, 32), dtype=np.uint8)
    dr = rng.integers(0, 256, (n_right, 32), dtype=np.uint8)
    npair = int(pair_frac * min(n_left, n_right))
    li = rng.choice(n_left, npair, replace=False)
    ri = rng.choice(n_right, npair, replace=False)
    l2r = np.full(n_left, -1, np.int32)
    r2l = np.full(n_right, -1, np.int32)
    l2r[li] = ri
    r2l[ri] = li
    bits = np.unpackbits(dl[li], axis=1)
    bits ^= (rng.random(bits.shape) < 0.03).astype(np.uint8)
    dr[ri] = np.packbits(bits, axis=1)
    kr["octave"][ri] = kl["octave"][li]

    def aim(k, d, n):
        near = rng.random(n_mp) < 0.8
        src = rng.integers(0, n, n_mp)
        nd = int(dup * n_mp)
        if nd:
            src[-nd:] = src[rng.integers(0, n_mp - nd, nd)]
        px = np.where(near, k["x"][src] + rng.normal(0, 1.5, n_mp), rng.uniform(0, W, n_mp)).astype(np.float32)
        py = np.where(near, k["y"][src] + rng.normal(0, 1.5, n_mp), rng.uniform(0, H, n_mp)).astype(np.float32)
        vc = np.where(rng.random(n_mp) < 0.5, rng.uniform(0.999, 1.0, n_mp), rng.uniform(0.5, 0.998, n_mp))
        lvl = np.clip(np.where(near, k["octave"][src] + rng.integers(-1, 2, n_mp), rng.integers(0, 8, n_mp)), 0, 7)
        return src, near, np.stack([px, py, np.zeros(n_mp), vc], 1).astype(np.float32), lvl.astype(np.int32)
    srcl, nearl, prl, lvl = aim(kl, dl, n_left)
    srcr, nearr, prr, lvr = aim(kr, dr, n_right)
    side = rng.random(n_mp)  # left only / right only / both
    bl = side < 0.75
    br = side > 0.45
    # a MapPoint seen in both images aims at a stereo pair's two keypoints when its left target has one
    both = bl & br & (l2r[srcl] >= 0)
    srcr = np.where(both, l2r[srcl], srcr)
    prr[both, 0] = kr["x"][srcr[both]] + rng.normal(0, 1.5, both.sum()).astype(np.float32)
    prr[both, 1] = kr["y"][srcr[both]] + rng.normal(0, 1.5, both.sum()).astype(np.float32)
    nearr = nearr | both
    lvr = np.where(both, np.clip(kr["octave"][srcr] + rng.integers(-1, 2, n_mp), 0, 7), lvr).astype(np.int32)
    lvr = np.where(rng.random(n_mp) < 0.05, -1, lvr).astype(np.int32)
    base = np.where(bl, dl[srcl].T, dr[srcr].T).T
    bits = np.unpackbits(base, axis=1)
    bits ^= (rng.random(bits.shape) < 0.06).astype(np.uint8)
    md = np.where((nearl | nearr)[:, None], np.packbits(bits, axis=1),
                  rng.integers(0, 256, (n_mp, 32), dtype=np.uint8))
    alive = rng.random(n_mp) < 0.92
    obs = rng.random(n_mp) < 0.85
    flags = ((bl & alive).astype(np.uint8) | (obs.astype(np.uint8) << 1) | ((br & alive).astype(np.uint8) << 2))
    return {"kps": kl, "desc": dl, "kps_r": kr, "desc_r": dr, "l2r": l2r, "r2l": r2l,
            "blocked": (rng.random(n_left) < 0.04).astype(np.uint8),
            "blocked_r": (rng.random(n_right) < 0.04).astype(np.uint8),
            "grid": grid_geometry(W, H), "scale_factors": orb_scale_factors(),
            "mp_flags": flags, "mp_proj": prl, "mp_level": lvl, "mp_proj_r": prr, "mp_level_r": lvr,
            "mp_desc": md.astype(np.uint8)}


def local_params(case, th):
    import plvi
    p = plvi.LocalParams()
    min_x, _, min_y, _, inv_w, inv_h = case["grid"]
    p.min_x, p.min_y, p.inv_w, p.inv_h, p.th, p.nlevels = min_x, min_y, inv_w, inv_h, th, 8
    for i, s in enumerate(case["scale_factors"]):
        p.scale_factors[i] = s
    return p


def line_proj_case(seed, n_cur=200, n_last=180, W=640, H=480, cols=64, rows=48):
    """Synthetic LineMatcher::SearchByProjection input: current-frame lines rasterised into the 64 x 48
    grid_Line with LineIterator (angles = atan2f of their endpoints, as KeyLine.angle), last-frame MapLines
    whose camera-frame endpoints project near a current line's (80 %) or anywhere, descriptors = the
    line's with ~8 % bit flips, duplicates aiming at the same current line (blocking order), some outliers
    / behind the camera / Observations() == 0, a few current lines pre-blocked."""
    rng = np.random.default_rng(seed)
    inv_w, inv_h = cols / W, rows / H
    sp = np.stack([rng.uniform(0, W - 1, n_cur), rng.uniform(0, H - 1, n_cur)], 1)
    ang = rng.uniform(0, 2 * np.pi, n_cur)
    ln = rng.uniform(10, 150, n_cur)
    ep = np.clip(sp + np.stack([np.cos(ang), np.sin(ang)], 1) * ln[:, None], 0, [W - 1, H - 1])
    sp32, ep32 = sp.astype(np.float32), ep.astype(np.float32)
    cur_angle = np.arctan2(ep32[:, 1] - sp32[:, 1], ep32[:, 0] - sp32[:, 0]).astype(np.float32)
    grid = [[[] for _ in range(rows)] for _ in range(cols)]
    for i in range(n_cur):
        for (x, y) in line_iterator(sp[i, 0] * inv_w, sp[i, 1] * inv_h, ep[i, 0] * inv_w, ep[i, 1] * inv_h):
            if 0 <= x < cols and 0 <= y < rows:
                grid[x][y].append(i)
    cur_desc = rng.integers(0, 256, (n_cur, 32), dtype=np.uint8)
    fx, fy, cx, cy = np.float32(458.654), np.float32(457.296), np.float32(320.0), np.float32(240.0)
    near = rng.random(n_last) < 0.8
    src = rng.integers(0, n_cur, n_last)
    k = n_last // 8
    src[-k:] = src[:k]
    x3 = np.zeros((n_last, 6), np.float32)
    for i in range(n_last):
        for e, P in enumerate((sp, ep)):
            u, v = (P[src[i]] + rng.normal(0, 1.0, 2)) if near[i] else rng.uniform([0, 0], [W, H])
            z = rng.uniform(1.0, 15.0)
            x3[i, 3 * e:3 * e + 3] = ((u - cx) * z / fx, (v - cy) * z / fy, z)
    x3[rng.random(n_last) < 0.03, 2] *= -1
    bits = np.unpackbits(cur_desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < 0.08).astype(np.uint8)
    ml = np.where(near[:, None], np.packbits(bits, axis=1), rng.integers(0, 256, (n_last, 32), dtype=np.uint8))
    flags = ((rng.random(n_last) < 0.92).astype(np.uint8) | ((rng.random(n_last) < 0.85).astype(np.uint8) << 1))
    return {"cur_angle": cur_angle, "cur_desc": cur_desc, "cur_blocked": (rng.random(n_cur) < 0.05).astype(np.uint8),
            "grid": grid, "last_flags": flags, "x3dc": x3,
            "last_octave": (rng.random(n_last) < 0.3).astype(np.int32), "ml_desc": ml.astype(np.uint8),
            "scale_l": np.array([1, 2, 0, 0, 0, 0, 0, 0], np.float32), "camera": (fx, fy, cx, cy),
            "bounds": (np.float32(0), np.float32(W), np.float32(0), np.float32(H)), "inv_w": inv_w, "inv_h": inv_h}


def line_proj_params(case, th, angth, range_hint=1):
    import plvi
    p = plvi.LineProjParams()
    p.fx, p.fy, p.cx, p.cy = case["camera"]
    p.min_x, p.max_x, p.min_y, p.max_y = case["bounds"]
    p.inv_w, p.inv_h, p.th, p.angth, p.range_hint, p.nlevels = case["inv_w"], case["inv_h"], th, angth, range_hint, 2
    for i, s in enumerate(case["scale_l"]):
        p.scale_l[i] = s
    return p


def proj_params(case, th, forward=0, backward=0):
    import plvi
    p = plvi.ProjParams()
    fx, fy, cx, cy, mbf = case["camera"]
    p.fx, p.fy, p.cx, p.cy, p.mbf, p.th = fx, fy, cx, cy, mbf, th
    (p.min_x, p.max_x, p.min_y, p.max_y, p.inv_w, p.inv_h) = case["grid"]
    p.forward, p.backward, p.nlevels = forward, backward, 8
    for i, s in enumerate(case["scale_factors"]):
        p.scale_factors[i] = s
    return p


def structured_frames(w=640, h=480):
    """Extreme-contrast 640x480 cases: a 0/255 vertical step, a 0/255
    checkerboard of 40-pixel squares, 3-pixel diagonal stripes and binary
    (0/255) noise -- gradients at the u8 maximum, lines running into the
    image border, and FAST / region-growing thresholds met almost everywhere."""
    yy, xx = np.mgrid[0:h, 0:w]
    out = {}
    out["step"] = np.where(xx < w // 2 + 3, 0, 255).astype(np.uint8)
    out["checker"] = np.where(((xx // 40) + (yy // 40)) % 2 == 0, 0, 255).astype(np.uint8)
    out["stripes"] = np.where(((xx + yy) // 3) % 2 == 0, 30, 220).astype(np.uint8)
    rng = np.random.default_rng(11)
    out["binary_noise"] = (rng.integers(0, 2, size=(h, w)) * 255).astype(np.uint8)
    return out


# Exact fused multiply-add (Python 3.10 has no math.fma): the reference build
# fuses some `a*b + c` sites (oracle/ref_fma.h, tests/test_ref_objects.py);
# the pure-Python restatements use these at the same sites.
def fma(a, b, c):
    """a*b + c rounded once to double (float(Fraction) is correctly rounded)."""
    from fractions import Fraction
    return float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def fmaf(a, b, c):
    """a*b + c on float32 operands rounded once to float32 (ties to even)."""
    from fractions import Fraction
    exact = Fraction(float(np.float32(a))) * Fraction(float(np.float32(b))) + Fraction(float(np.float32(c)))
    f = np.float32(float(exact))  # double then float32: may double-round, fixed below
    best = f
    for g in (np.nextafter(f, np.float32(-np.inf)), np.nextafter(f, np.float32(np.inf))):
        dg, db = abs(Fraction(float(g)) - exact), abs(Fraction(float(best)) - exact)
        if dg < db or (dg == db and (int(np.float32(g).view(np.uint32)) & 1) == 0):
            best = g
    return np.float32(best)


# ------------------------------------------------------------- frustum cases
def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def frustum_params(seed, model=0, two_camera=False, far_points=False, compat=0, nlevels=8, scale=1.2):
    """plvi_frustum_params of a synthetic frame: random pose (Rcw, tcw, Ow = -Rcw^T tcw as float), EuRoC-like
    Pinhole (752 x 480, mbf = 0.11 fx) or TUM-VI-like KannalaBrandt8 (512 x 512); two_camera adds a right
    camera 0.1 m to the side (R = Rrl Rcw, t = Rrl tcw + trl, O = Rwc tlr + Ow) with a slight rotation."""
    import plvi
    rng = np.random.default_rng(seed)
    p = plvi.FrustumParams()
    R = _rotation(rng)
    t = rng.normal(0, 2, 3)
    Ow = -R.T @ t

    def set_cam(c, R_, t_, O_):
        for i in range(9):
            c.R[i] = np.float32(R_.flat[i])
        for i in range(3):
            c.t[i] = np.float32(t_[i])
            c.O[i] = np.float32(O_[i])
        if model == 0:
            c.fx, c.fy, c.cx, c.cy = 458.654, 457.296, 367.215, 248.375
        else:
            c.fx, c.fy, c.cx, c.cy = (float(v) for v in KB8_TUMVI[:4])
            for i in range(4):
                c.kb[i] = KB8_TUMVI[4 + i]
        c.model = model

    set_cam(p.cam[0], R, t, Ow)
    if two_camera:
        a = 0.02
        Rrl = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        trl = np.array([-0.101, 0.002, 0.001])
        tlr = -Rrl.T @ trl
        set_cam(p.cam[1], Rrl @ R, Rrl @ t + trl, R.T @ tlr + Ow)
    p.two_camera = int(two_camera)
    p.mbf = np.float32(0.11) * np.float32(p.cam[0].fx) if model == 0 else 0.0
    if model == 0:
        p.min_x, p.max_x, p.min_y, p.max_y = -0.75, 752.5, 0.25, 479.25
    else:
        p.min_x, p.max_x, p.min_y, p.max_y = 0.0, 512.0, 0.0, 512.0
    p.view_cos_limit = 0.5
    p.far_points, p.far_th = int(far_points), 9.0
    p.nlevels = nlevels
    p.log_scale_factor = float(np.float32(np.log(np.float32(scale))))
    p.compat = compat
    plvi.frustum_params_init(p)
    return p


def _cam_points(rng, n, model):
    """Camera-frame points: most in front and inside / around the field of view, some behind."""
    z = np.where(rng.random(n) < 0.1, rng.uniform(-3, 0, n), rng.uniform(0.05, 25, n))
    s = 0.9 if model == 0 else 2.5
    return np.stack([z * rng.uniform(-s, s, n), z * rng.uniform(-s * 0.7, s * 0.7, n), z], 1)


def _world(p, pc, cam=0):
    c = p.cam[cam]
    R = np.array(c.R[:], np.float64).reshape(3, 3)
    t = np.array(c.t[:], np.float64)
    return (pc - t) @ R  # R^T (pc - t)


def _normals(rng, po):
    """Unit normals at ~0-90 degrees from the viewing ray PO (the view cos straddles 0.5)."""
    u = po / np.maximum(np.linalg.norm(po, axis=1, keepdims=True), 1e-12)
    perp = np.cross(u, rng.normal(size=u.shape))
    perp /= np.maximum(np.linalg.norm(perp, axis=1, keepdims=True), 1e-12)
    a = rng.uniform(0, np.pi / 2, len(u))
    return (u * np.cos(a)[:, None] + perp * np.sin(a)[:, None]).astype(np.float32)


def frustum_case(seed, p, n=3000):
    """Local MapPoints of frame p (Tracking::SearchLocalPoints input): world positions, normals, {mfMinDistance,
    mfMaxDistance} straddling the 0.8 / 1.2 invariance bounds with max/dist ratios over every level, flags,
    and stale MapPoint fields from an earlier frame; plus degenerate points (camera centre, zero depth)."""
    rng = np.random.default_rng(seed)
    model = p.cam[0].model
    pw = _world(p, _cam_points(rng, n, model)).astype(np.float32)
    O = np.array(p.cam[0].O[:], np.float32)
    d = np.linalg.norm(pw.astype(np.float64) - O, axis=1)
    mx = d * 1.2 ** rng.uniform(-1.3, 8.5, n)
    mn = d / 0.8 * 1.2 ** rng.uniform(-8, 0.4, n)
    # degenerate: the camera centre itself (Pc ~ 0, dist 0), zero max / min distance
    pw[:4] = O
    mx[:2], mn[:4] = 0.0, 0.0
    dist = np.stack([mn, mx], 1).astype(np.float32)
    case = {"pos": pw, "normal": _normals(rng, pw.astype(np.float64) - O), "dist": dist,
            "in_flags": ((rng.random(n) < 0.9).astype(np.uint8) | ((rng.random(n) < 0.85).astype(np.uint8) << 1)),
            "proj": rng.uniform(-5, 800, (n, 4)).astype(np.float32), "level": rng.integers(-1, 8, n).astype(np.int32),
            "depth": rng.uniform(0, 30, n).astype(np.float32),
            "proj_r": rng.uniform(-5, 800, (n, 4)).astype(np.float32),
            "level_r": rng.integers(-1, 8, n).astype(np.int32)}
    case["in_flags"][:4] |= 1
    return case


def frustum_line_case(seed, p, n=800):
    """Local MapLines of frame p: world endpoints (double) of segments in front / behind / across the image
    border, float normals, {mfMinDistance, mfMaxDistance}, evaluated flags, descriptors, stale fields."""
    rng = np.random.default_rng(seed)
    a = _cam_points(rng, n, 0)
    b = a + rng.normal(0, 1.0, (n, 3)) * np.maximum(a[:, 2:3], 0.5) * 0.3
    sp, ep = _world(p, a), _world(p, b)
    O = np.array(p.cam[0].O[:], np.float64)
    mid = (sp + ep) / 2 - O
    d = np.linalg.norm(mid, axis=1)
    dist = np.stack([d / 0.8 * 1.2 ** rng.uniform(-6, 0.4, n), d * 1.2 ** rng.uniform(-1.3, 6, n)], 1)
    return {"sep": np.concatenate([sp, ep], 1), "normal": _normals(rng, mid), "dist": dist.astype(np.float32),
            "in_flags": (rng.random(n) < 0.9).astype(np.uint8),
            "desc": rng.integers(0, 256, (n, 32), dtype=np.uint8),
            "proj": rng.uniform(-5, 800, (n, 4)).astype(np.float32), "angle": rng.uniform(-3, 3, n)}
