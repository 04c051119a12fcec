"""ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) with a two-camera
CurrentFrame (CurrentFrame.Nleft != -1, src/ORBmatcher.cc:1985-2175): every LastFrame point is projected by
CurrentFrame.mpCamera (KannalaBrandt8::project, CameraModels/KannalaBrandt8.cpp:33-48, or Pinhole) into the
left image and -- unless the left pass ended early -- into the right image (x3Dr = mTrl x3Dc, mGridRight);
both images' matches share one rotation histogram.

Parity unpinned: the reference has no tests for it.  The C++ oracle (oracle/proj_oracle.cpp:
oracle_search_by_projection2, host libm for atan2f / cosf / sinf as the reference calls them) restates the
cited lines; with a Pinhole rig it is checked here against the one-camera oracle on a frame whose right image
is empty, and its KannalaBrandt8 projection against a float64 model; the HIP path (search_by_projection2_kernel,
csrc/proj.hip, glibc atan2f / cosf / sinf restated in csrc/plvi_math.h) is compared with the oracle exactly
(both match tables incl. overwrites and the rotation filter's NULLs, nmatches)."""
import numpy as np
import pytest

import oracle_lib
import util


def test_oracle_stereo_projection_reduces_to_one_camera():
    """Pinhole rig, empty right image: the two-camera restatement equals the one-camera oracle."""
    c = util.projection_stereo_case(1, kb8=False)
    c["kps_r"], c["desc_r"], c["blocked_r"] = c["kps_r"][:0], c["desc_r"][:0], c["blocked_r"][:0]
    n2, ml, mr = oracle_lib.search_by_projection_stereo(c, 7.0)
    mono = {"cur_kps": c["kps"], "cur_desc": c["desc"], "cur_blocked": c["blocked"], "cur_uright": None,
            "grid": c["grid"], "scale_factors": c["scale_factors"], "x3dc": c["x3dc"], "flags": c["flags"],
            "last_octave": c["last_octave"], "last_angle": c["last_angle"], "mp_desc": c["mp_desc"],
            "camera": c["camera"]}
    n1, m1 = oracle_lib.search_by_projection(mono, 7.0)
    assert n2 == n1 and len(mr) == 0
    np.testing.assert_array_equal(ml, m1)
    assert n1 > 100


def test_oracle_stereo_projection_sanity():
    c = util.projection_stereo_case(2)
    n, ml, mr = oracle_lib.search_by_projection_stereo(c, 7.0)
    assert (ml >= 0).sum() > 150 and (mr >= 0).sum() > 80  # both images match
    assert (ml == -2).sum() + (mr == -2).sum() > 0          # the shared rotation filter bites
    assert n > 0 and n <= (ml != -1).sum() + (mr != -1).sum() + 200  # overwrites count in nmatches
    # Pinhole instead of KannalaBrandt8 on the same points: a different (fewer-match) answer, so the
    # fisheye projection is really used
    d = dict(c)
    d["kb8"] = None
    n0, ml0, _ = oracle_lib.search_by_projection_stereo(d, 7.0)
    assert not np.array_equal(ml0, ml)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,kb8,fb", [(0, 7.0, True, (0, 0)), (1, 15.0, True, (0, 0)), (2, 7.0, False, (0, 0)),
                                            (3, 7.0, True, (1, 0)), (4, 7.0, True, (0, 1)), (5, 3.0, True, (0, 0))])
def test_stereo_projection_matches_oracle(seed, th, kb8, fb):
    import plvi
    c = util.projection_stereo_case(30 + seed, kb8=kb8)
    ne, mle, mre = oracle_lib.search_by_projection_stereo(c, th, forward=fb[0], backward=fb[1])
    ng, mlg, mrg = plvi.ORBmatcher(0.9, True).SearchByProjectionStereo(
        util.proj_params(c, th, *fb), c["kps"], c["desc"], c["kps_r"], c["desc_r"], c["x3dc"], c["x3dr"],
        c["last_octave"], c["last_angle"], c["mp_desc"], c["flags"], c["kb8"], c["blocked"], c["blocked_r"])
    assert ng == ne
    np.testing.assert_array_equal(mlg, mle)
    np.testing.assert_array_equal(mrg, mre)


@pytest.mark.gpu
def test_stereo_projection_no_rotation_check_and_degenerate():
    import plvi
    c = util.projection_stereo_case(40)
    ne, mle, mre = oracle_lib.search_by_projection_stereo(c, 7.0, check_ori=0)
    ng, mlg, mrg = plvi.ORBmatcher(0.9, False).SearchByProjectionStereo(
        util.proj_params(c, 7.0), c["kps"], c["desc"], c["kps_r"], c["desc_r"], c["x3dc"], c["x3dr"],
        c["last_octave"], c["last_angle"], c["mp_desc"], c["flags"], c["kb8"], c["blocked"], c["blocked_r"])
    assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre)
    mt = plvi.ORBmatcher(0.9, True)
    for cut in ("last", "right", "left"):
        d = dict(c)
        if cut == "last":
            for k in ("x3dc", "x3dr", "flags", "last_octave", "last_angle", "mp_desc"):
                d[k] = c[k][:0]
        elif cut == "right":
            d["kps_r"], d["desc_r"], d["blocked_r"] = c["kps_r"][:0], c["desc_r"][:0], c["blocked_r"][:0]
        else:
            d["kps"], d["desc"], d["blocked"] = c["kps"][:0], c["desc"][:0], c["blocked"][:0]
        ne, mle, mre = oracle_lib.search_by_projection_stereo(d, 7.0)
        ng, mlg, mrg = mt.SearchByProjectionStereo(
            util.proj_params(d, 7.0), d["kps"], d["desc"], d["kps_r"], d["desc_r"], d["x3dc"], d["x3dr"],
            d["last_octave"], d["last_angle"], d["mp_desc"], d["flags"], d["kb8"], d["blocked"], d["blocked_r"])
        assert ng == ne and np.array_equal(mlg, mle) and np.array_equal(mrg, mre), cut
