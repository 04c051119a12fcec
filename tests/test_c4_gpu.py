"""BASELINE C4 at its own shape: a 752x480 EuRoC-shaped sequence window
(seeds s*10^6 + t, the shard of rank s) through the bench's step --
plvi_frame_extract_batch (Frame::Frame's ORB || LSD/LBD, src/Frame.cc:537-692),
ORB kNN-2 of every frame against its predecessor and LineMatcher::match
(src/LineMatcher.cpp:88-111) -- with the first, middle and last frames and a
consecutive pair compared bit-exactly with the oracle; and the per-step
table gather (plvi.dist.TableGather) staging exactly the extractor tables
(Examples/Monocular-Inertial/mono_inertial_euroc.cc:40,175 walk one sequence)."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import dist as pdist
from plvi import synth

pytestmark = pytest.mark.gpu

W, H = 752, 480


def test_c4_sequence_window_vs_oracle():
    import torch
    n = 256
    seq = synth.device_sequence(n, W, H, seed=pdist.shard_seed(1), device="cuda:0")
    torch.cuda.synchronize()
    lib = plvi.load()
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=n)
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=n)
    kp, de, co, mo, cap = orb.outputs()
    kl, lde, fn, lco, lcap = lx.outputs()
    i32 = dict(dtype=torch.int32, device="cuda:0")
    outs = [torch.full(((n - 1) * cap,), -7, **i32) for _ in range(4)]
    lsc = torch.empty(4 * (n - 1) * 2 * lcap, **i32)
    lm12 = torch.full(((n - 1) * lcap,), -7, **i32)
    lnm = torch.empty(n - 1, **i32)
    s = torch.cuda.Stream()
    st = s.cuda_stream
    plvi.frame_extract_batch(orb, lx, seq.data_ptr(), n, W * H, W, (0, 0), stream=st)
    assert lib.plvi_hamming_knn2_batch(de + cap * 32, co + 4, cap, de, co, cap, n - 1,
                                       *[o.data_ptr() for o in outs], st) == 0
    assert lib.plvi_line_match_batch(lde + lcap * 32, lco + 4, lcap, lde, lco, lcap, n - 1, 0.9, lsc.data_ptr(),
                                     lm12.data_ptr(), lnm.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert orb.errors(st) == 0 and lx.errors(st) == 0
    cnt = plvi.download(co, np.zeros(n, np.int32))
    mono = plvi.download(mo, np.zeros(n, np.int32))
    lcnt = plvi.download(lco, np.zeros(n, np.int32))
    tabs = {}
    p = n // 2 - 1
    for f in (0, p, p + 1, n - 1):
        k = plvi.download(kp + 28 * cap * f, np.zeros(int(cnt[f]), plvi.KEYPOINT_DTYPE))
        d = plvi.download(de + 32 * cap * f, np.zeros((int(cnt[f]), 32), np.uint8))
        ln = plvi.download(kl + 68 * lcap * f, np.zeros(int(lcnt[f]), plvi.KEYLINE_DTYPE))
        ld = plvi.download(lde + 32 * lcap * f, np.zeros((int(lcnt[f]), 32), np.uint8))
        lf = plvi.download(fn + 24 * lcap * f, np.zeros((int(lcnt[f]), 3), np.float64))
        tabs[f] = (d, ld)
        img = seq[f].cpu().numpy()
        m, ek, ed = ol.orb_extract(img)
        assert int(mono[f]) == m and len(ek) > 300, f"frame {f}"
        assert k.tobytes() == ek.astype(plvi.KEYPOINT_DTYPE).tobytes(), f"frame {f} keypoints"
        np.testing.assert_array_equal(d, ed)
        ekl, eld, efn = ol.line_extract(img)
        assert len(ekl) > 20, f"frame {f}"
        assert ln.tobytes() == ekl.astype(plvi.KEYLINE_DTYPE).tobytes(), f"frame {f} keylines"
        np.testing.assert_array_equal(ld, eld)
        assert lf.tobytes() == efn.tobytes()
    # pair p: frame p+1 (query) against frame p (train)
    n1 = int(cnt[p + 1])
    got = [o[cap * p:cap * p + n1].cpu().numpy() for o in outs]
    exp = ol.knn2(tabs[p + 1][0], tabs[p][0])
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)
    nm, m12 = ol.match(tabs[p + 1][1], tabs[p][1], 0.9)
    assert int(lnm[p]) == nm
    np.testing.assert_array_equal(lm12[lcap * p:lcap * p + len(tabs[p + 1][1])].cpu().numpy(), m12)

    # the bench's timed gather staging: world 1 stages on the step's stream
    sizes = (4 * n, 28 * cap * n, 32 * cap * n, 4 * n, 68 * lcap * n, 32 * lcap * n)

    def dev_copy(t, src):
        assert lib.plvi_memcpy_async(t.data_ptr(), src, t.numel(), 3, st) == 0
    tg = pdist.TableGather(sizes, 1, 0, device="cuda:0", copy=dev_copy)
    tg.post((co, kp, de, lco, kl, lde), stream=s)
    tg.wait()
    torch.cuda.synchronize()
    staged = tg.received(0)
    for t, src in zip(staged, (co, kp, de, lco, kl, lde)):
        assert np.array_equal(t.cpu().numpy(), plvi.download(src, np.zeros(t.numel(), np.uint8)))
