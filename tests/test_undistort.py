"""Frame::UndistortKeyPoints / UndistortKeyLines / ComputeImageBounds
(src/Frame.cc:1124-1226) = cv::undistortPoints (OpenCV 4.2, 5 iterations,
R = I, P = K), SURVEY §8f rank 3.

Parity unpinned: OpenCV is absent from this image; the oracle restates
cvUndistortPointsInternal and is cross-checked against a numpy restatement
and a distort -> undistort round trip; the HIP path is compared with the
oracle bit-exactly."""
import numpy as np
import pytest

import oracle_lib

# EuRoC cam0 (Examples/Monocular/EuRoC.yaml shape): fx fy cx cy, k1 k2 p1 p2
K_EUROC = np.array([458.654, 457.296, 367.215, 248.375], np.float32)
D_EUROC = np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32)
D_K3 = np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0123], np.float32)


def py_undistort(K, D, xy):
    fx, fy, cx, cy = (float(v) for v in K)
    k = [float(v) for v in D] + [0.0] * (14 - len(D))
    out = []
    for sx, sy in xy:
        x = (float(sx) - cx) * (1.0 / fx)
        y = (float(sy) - cy) * (1.0 / fy)
        x0, y0 = x, y
        for _ in range(5):
            r2 = x * x + y * y
            icd = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
            x = (x0 - dx) * icd
            y = (y0 - dy) * icd
        out.append((np.float32(fx * x + 0.0 * y + cx), np.float32(0.0 * x + fy * y + cy)))
    return np.array(out, np.float32)


def distort(K, D, xy):
    fx, fy, cx, cy = (float(v) for v in K)
    k1, k2, p1, p2 = (float(v) for v in D[:4])
    k3 = float(D[4]) if len(D) > 4 else 0.0
    x = (xy[:, 0].astype(np.float64) - cx) / fx
    y = (xy[:, 1].astype(np.float64) - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


def _pts(seed, n, W=752, H=480):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(0, W, n), rng.uniform(0, H, n)], 1).astype(np.float32)


@pytest.mark.parametrize("D", [D_EUROC, D_K3])
def test_oracle_matches_numpy_restatement(D):
    xy = _pts(1, 300)
    np.testing.assert_array_equal(oracle_lib.undistort_points(K_EUROC, D, xy), py_undistort(K_EUROC, D, xy))


def test_oracle_round_trip_and_identity():
    xy = _pts(2, 500, 600, 400) + np.float32([76, 40])   # central region: 5 iterations converge
    und = oracle_lib.undistort_points(K_EUROC, D_EUROC, xy)
    back = distort(K_EUROC, D_EUROC, und)
    err = np.abs(back - xy).max(1)
    assert np.median(err) < 0.01 and err.max() < 0.5  # 5 fixed-point iterations: not fully converged at the rim
    z = np.zeros(4, np.float32)
    np.testing.assert_array_equal(oracle_lib.undistort_points(K_EUROC, z, xy), xy)  # mDistCoef(0) == 0: copy
    b = oracle_lib.image_bounds(K_EUROC, D_EUROC, 752, 480)
    assert b[0] < 0 and b[1] > 752 and b[2] < 0 and b[3] > 480   # barrel distortion widens the bounds
    np.testing.assert_array_equal(oracle_lib.image_bounds(K_EUROC, z, 752, 480), [0, 752, 0, 480])


@pytest.mark.gpu
@pytest.mark.parametrize("D", [D_EUROC, D_K3, np.zeros(4, np.float32)])
def test_undistort_points_matches_oracle(D):
    import plvi
    cam = plvi.Camera.make(*K_EUROC, D)
    xy = np.concatenate([_pts(3, 4000), np.float32([[0, 0], [752, 0], [0, 480], [752, 480], [-20, 500]])])
    np.testing.assert_array_equal(plvi.undistort_points(cam, xy), oracle_lib.undistort_points(K_EUROC, D, xy))
    np.testing.assert_array_equal(plvi.image_bounds(cam, 752, 480), oracle_lib.image_bounds(K_EUROC, D, 752, 480))


@pytest.mark.gpu
def test_undistort_keypoint_and_keyline_tables():
    import ctypes
    import plvi
    lib = plvi.load()
    cam = plvi.Camera.make(*K_EUROC, D_EUROC)
    rng = np.random.default_rng(4)
    B, cap = 3, 600
    counts = np.array([600, 17, 350], np.int32)
    kp = np.zeros((B, cap), plvi.KEYPOINT_DTYPE)
    kp["x"] = rng.uniform(0, 752, (B, cap)); kp["y"] = rng.uniform(0, 480, (B, cap))
    kp["angle"] = rng.uniform(0, 360, (B, cap)); kp["octave"] = rng.integers(0, 8, (B, cap)); kp["size"] = 31
    kl = np.zeros((B, cap), plvi.KEYLINE_DTYPE)
    for f in ("startPointX", "endPointX"):
        kl[f] = rng.uniform(0, 752, (B, cap))
    for f in ("startPointY", "endPointY"):
        kl[f] = rng.uniform(0, 480, (B, cap))
    bufs = []

    def dev(a):
        b = plvi.DeviceBuffer(a.nbytes); b.upload(np.ascontiguousarray(a)); bufs.append(b)
        return ctypes.c_void_p(b.ptr)
    ok = plvi.DeviceBuffer(kp.nbytes); oe = plvi.DeviceBuffer(B * cap * 16)
    dc = dev(counts)
    assert lib.plvi_undistort_keypoints_batch(ctypes.byref(cam), dev(kp), dc, cap, B, ctypes.c_void_p(ok.ptr),
                                              None) == 0
    assert lib.plvi_undistort_keylines_batch(ctypes.byref(cam), dev(kl), dc, cap, B, ctypes.c_void_p(oe.ptr),
                                             None) == 0
    lib.plvi_device_synchronize()
    gk = ok.download(np.zeros((B, cap), plvi.KEYPOINT_DTYPE))
    ge = oe.download(np.zeros((B, cap, 4), np.float32))
    for f in range(B):
        n = counts[f]
        exp = oracle_lib.undistort_points(K_EUROC, D_EUROC, np.stack([kp["x"][f, :n], kp["y"][f, :n]], 1))
        np.testing.assert_array_equal(gk["x"][f, :n], exp[:, 0])
        np.testing.assert_array_equal(gk["y"][f, :n], exp[:, 1])
        for fld in ("angle", "octave", "size", "response", "class_id"):
            np.testing.assert_array_equal(gk[fld][f, :n], kp[fld][f, :n])
        s = oracle_lib.undistort_points(K_EUROC, D_EUROC, np.stack([kl["startPointX"][f, :n], kl["startPointY"][f, :n]], 1))
        e = oracle_lib.undistort_points(K_EUROC, D_EUROC, np.stack([kl["endPointX"][f, :n], kl["endPointY"][f, :n]], 1))
        np.testing.assert_array_equal(ge[f, :n], np.concatenate([s, e], 1))
