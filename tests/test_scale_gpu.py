"""Parity at the configurations BASELINE.json quotes, not just at
toy sizes:

  C1/C2: plvi_frame_extract_batch over a batch of 64 synthetic 640x480
         frames (ORB || LSD+LBD in one schedule), every frame vs the oracle;
  C3:    plvi_hamming_knn2_batch over 256 independent 1000x1000 pairs of
         256-bit descriptors (60 % near-duplicates, Binomial(256, 0.08)
         flips) and plvi_line_match_batch over 256 pairs of 200x200 LBD-sized
         tables, every pair vs the oracle (BFMatcher tie rules, ratio 0.9,
         mutual check).
"""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import near_duplicate_descriptors

pytestmark = pytest.mark.gpu


def test_c1c2_frame_batch_64(plvi_lib):
    B = 64
    frames = synth.batch(B, seed0=1000)
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
    buf = plvi.DeviceBuffer(frames.nbytes)
    buf.upload(frames)
    plvi.frame_extract_batch(orb, lx, buf.ptr, B, 640 * 480, 640, (0, 0))
    plvi_lib.plvi_device_synchronize()
    assert orb.errors() == 0 and lx.errors() == 0
    kp_p, de_p, co_p, mo_p, cap = orb.outputs()
    cnt = plvi.download(co_p, np.zeros(B, np.int32))
    mono = plvi.download(mo_p, np.zeros(B, np.int32))
    kps = plvi.download(kp_p, np.zeros(B * cap, plvi.KEYPOINT_DTYPE))
    desc = plvi.download(de_p, np.zeros((B * cap, 32), np.uint8))
    klp, ldp, fnp, lcop, lcap = lx.outputs()
    lcnt = plvi.download(lcop, np.zeros(B, np.int32))
    kl = plvi.download(klp, np.zeros(B * lcap, plvi.KEYLINE_DTYPE))
    ld = plvi.download(ldp, np.zeros((B * lcap, 32), np.uint8))
    fn = plvi.download(fnp, np.zeros((B * lcap, 3), np.float64))
    bad = []
    for f in range(B):
        m, k, d = ol.orb_extract(frames[f])
        s = slice(f * cap, f * cap + cnt[f])
        if not (mono[f] == m and kps[s].tobytes() == k.tobytes() and np.array_equal(desc[s], d)):
            bad.append(("orb", f))
        k2, d2, f2 = ol.line_extract(frames[f])
        s = slice(f * lcap, f * lcap + lcnt[f])
        if not (kl[s].tobytes() == k2.tobytes() and np.array_equal(ld[s], d2) and fn[s].tobytes() == f2.tobytes()):
            bad.append(("lines", f))
    assert not bad, bad[:10]


def _upload(**arrays):
    bufs = {}
    for k, v in arrays.items():
        bufs[k] = plvi.DeviceBuffer(v.nbytes)
        bufs[k].upload(v)
    return bufs


def test_c3_knn2_256_pairs_1000x1000(plvi_lib):
    P, N = 256, 1000
    rng = np.random.default_rng(33)
    q = np.zeros((P, N, 32), np.uint8)
    t = np.zeros((P, N, 32), np.uint8)
    for p in range(P):
        q[p], t[p] = near_duplicate_descriptors(rng, N, N)
    nq = np.full(P, N, np.int32)
    nt = np.full(P, N, np.int32)
    nq[7], nt[9], nt[11] = 0, 1, 0  # degenerate pairs inside the batch
    b = _upload(q=q, t=t, nq=nq, nt=nt)
    outs = [plvi.DeviceBuffer(P * N * 4) for _ in range(4)]
    rc = plvi_lib.plvi_hamming_knn2_batch(b["q"].ptr, b["nq"].ptr, N, b["t"].ptr, b["nt"].ptr, N, P,
                                          *[o.ptr for o in outs], None)
    assert rc == 0
    plvi_lib.plvi_device_synchronize()
    got = [o.download(np.zeros((P, N), np.int32)) for o in outs]
    for p in range(P):
        exp = ol.knn2(q[p, :nq[p]], t[p, :nt[p]])
        for g, e in zip(got, exp):
            assert np.array_equal(g[p, :nq[p]], e), p


def test_c3_line_match_256_pairs(plvi_lib):
    P, cap = 256, 200
    rng = np.random.default_rng(44)
    d1 = np.zeros((P, cap, 32), np.uint8)
    d2 = np.zeros((P, cap, 32), np.uint8)
    n1 = rng.integers(150, cap + 1, P).astype(np.int32)
    n2 = rng.integers(150, cap + 1, P).astype(np.int32)
    n2[3], n1[5] = 1, 0
    for p in range(P):
        a, bb = near_duplicate_descriptors(rng, max(int(n2[p]), 1), max(int(n1[p]), 1), p_flip=0.05)
        d1[p, :n1[p]] = a[:n1[p]]
        d2[p, :n2[p]] = bb[:n2[p]]
    b = _upload(d1=d1, d2=d2, n1=n1, n2=n2)
    scratch = plvi.DeviceBuffer(4 * P * 2 * cap * 4)
    m12 = plvi.DeviceBuffer(P * cap * 4)
    nm = plvi.DeviceBuffer(P * 4)
    rc = plvi_lib.plvi_line_match_batch(b["d1"].ptr, b["n1"].ptr, cap, b["d2"].ptr, b["n2"].ptr, cap, P, 0.9,
                                        scratch.ptr, m12.ptr, nm.ptr, None)
    assert rc == 0
    plvi_lib.plvi_device_synchronize()
    gm = m12.download(np.zeros((P, cap), np.int32))
    gn = nm.download(np.zeros(P, np.int32))
    for p in range(P):
        if n2[p] < 2:  # the reference indexes the second neighbour: the batch produces no matches
            assert gn[p] == 0 and (gm[p, :n1[p]] == -1).all()
            continue
        ne, me = ol.match(d1[p, :n1[p]], d2[p, :n2[p]], 0.9)
        assert gn[p] == ne and np.array_equal(gm[p, :n1[p]], me), p
