"""plvi — Python host mirror of the MI355X front end's C-ABI.

Thin ctypes layer over ``lib/libplvi_frontend.so`` (built from ``csrc/``).
Class and method names follow the reference interfaces they replace:

  ORBextractor  -> ORB_SLAM3::ORBextractor (include/ORBextractor.h:44-110)
  LineMatcher   -> ORB_SLAM3::LineMatcher  (include/LineMatcher.h:88-107)
  ORBmatcher    -> ORB_SLAM3::ORBmatcher   (include/ORBmatcher.h:39-68): SearchByBoW, DescriptorDistance
  hamming_knn2  -> cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) (LineMatcher.cpp:47-48)
  ORBVocabulary -> DBoW2::TemplatedVocabulary<FORB> (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h):
                   loadFromTextFile, transform(features, BowVector&, FeatureVector&, levelsup)

There is no CPU fallback: if the HIP library is missing or no GPU is
visible, construction raises.  PyTorch is only used by bench.py for device
memory and streams; this module needs numpy only.
"""
import ctypes
import os
import sys
import pathlib

import numpy as np

_PKG = pathlib.Path(__file__).resolve().parent.parent
# PLVI_LIB: an alternative build of the same library (A/B experiments, tools/build_variant.sh)
LIB_PATH = pathlib.Path(os.environ["PLVI_LIB"]) if os.environ.get("PLVI_LIB") else _PKG / "lib" / "libplvi_frontend.so"
HEADER_PATH = _PKG.parent / "include" / "plvi_frontend.h"

PLVI_OK = 0
PLVI_E_EMPTY = -1
PLVI_E_BADARG = -2
PLVI_E_CAPACITY = -3
PLVI_E_HIP = -4
PLVI_E_OVERFLOW = -5
PLVI_E_SIZE = -6
PLVI_E_CAPTURE = -7

# OpenCV-semantics switches (plvi_frontend.h PLVI_COMPAT_*)
COMPAT_GAUSS_ROUNDED = 1
COMPAT_RESIZE_V_GENERIC = 2
COMPAT_EXP_CV_TABLE = 4

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
KEYLINE_DTYPE = np.dtype([("angle", "<f4"), ("class_id", "<i4"), ("octave", "<i4"), ("pt_x", "<f4"),
                          ("pt_y", "<f4"), ("response", "<f4"), ("size", "<f4"), ("startPointX", "<f4"),
                          ("startPointY", "<f4"), ("endPointX", "<f4"), ("endPointY", "<f4"),
                          ("sPointInOctaveX", "<f4"), ("sPointInOctaveY", "<f4"), ("ePointInOctaveX", "<f4"),
                          ("ePointInOctaveY", "<f4"), ("lineLength", "<f4"), ("numOfPixels", "<i4")])


class PlviError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what} failed with status {code}")
        self.code = code


class GridParams(ctypes.Structure):
    """plvi_grid_params: mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv."""
    _fields_ = [("min_x", ctypes.c_float), ("min_y", ctypes.c_float), ("inv_w", ctypes.c_float),
                ("inv_h", ctypes.c_float)]


class Camera(ctypes.Structure):
    """plvi_camera: mK (fx, fy, cx, cy) and mDistCoef (k1, k2, p1, p2[, k3])."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("dist", ctypes.c_float * 5), ("ndist", ctypes.c_int)]

    @classmethod
    def make(cls, fx, fy, cx, cy, dist):
        c = cls()
        c.fx, c.fy, c.cx, c.cy = fx, fy, cx, cy
        for i, d in enumerate(dist):
            c.dist[i] = d
        c.ndist = len(dist)
        return c


def undistort_points(cam, xy):
    """cv::undistortPoints as Frame::UndistortKeyPoints calls it (src/Frame.cc:1124-1157): n x 2 float32."""
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    n = xy.shape[0]
    lib = load()
    d_in, d_out = DeviceBuffer(max(xy.nbytes, 8)), DeviceBuffer(max(xy.nbytes, 8))
    d_in.upload(xy)
    _check(lib.plvi_undistort_points(ctypes.byref(cam), ctypes.c_void_p(d_in.ptr), n, ctypes.c_void_p(d_out.ptr),
                                     None), "plvi_undistort_points")
    lib.plvi_device_synchronize()
    return d_out.download(np.zeros((n, 2), np.float32))


def image_bounds(cam, cols, rows):
    """Frame::ComputeImageBounds (src/Frame.cc:1199-1226): (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
    b = np.zeros(4, np.float32)
    _check(load().plvi_image_bounds(ctypes.byref(cam), cols, rows, _ptr(b)), "plvi_image_bounds")
    return b


class ProjParams(ctypes.Structure):
    """plvi_proj_params (include/plvi_frontend.h)."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("mbf", ctypes.c_float), ("th", ctypes.c_float), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("inv_w", ctypes.c_float), ("inv_h", ctypes.c_float), ("forward", ctypes.c_int),
                ("backward", ctypes.c_int), ("check_orientation", ctypes.c_int), ("nlevels", ctypes.c_int),
                ("scale_factors", ctypes.c_float * 16)]


class InitParams(ctypes.Structure):
    """plvi_init_params (include/plvi_frontend.h): ORBmatcher::SearchForInitialization."""
    _fields_ = [("min_x", ctypes.c_float), ("min_y", ctypes.c_float), ("inv_w", ctypes.c_float),
                ("inv_h", ctypes.c_float), ("window", ctypes.c_int), ("nnratio", ctypes.c_float),
                ("check_orientation", ctypes.c_int)]


class LocalParams(ctypes.Structure):
    """plvi_local_params (include/plvi_frontend.h): ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>...)."""
    _fields_ = [("min_x", ctypes.c_float), ("min_y", ctypes.c_float), ("inv_w", ctypes.c_float),
                ("inv_h", ctypes.c_float), ("th", ctypes.c_float), ("nnratio", ctypes.c_float),
                ("nlevels", ctypes.c_int), ("scale_factors", ctypes.c_float * 16)]


class RelocParams(ctypes.Structure):
    """plvi_reloc_params (include/plvi_frontend.h): ORBmatcher::SearchByProjection(Frame&, KeyFrame*,
    sAlreadyFound, th, ORBdist)."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float), ("min_y", ctypes.c_float),
                ("max_y", ctypes.c_float), ("inv_w", ctypes.c_float), ("inv_h", ctypes.c_float),
                ("th", ctypes.c_float), ("orb_dist", ctypes.c_int), ("check_orientation", ctypes.c_int),
                ("nlevels", ctypes.c_int), ("scale_factors", ctypes.c_float * 16)]


class LineProjParams(ctypes.Structure):
    """plvi_line_proj_params (include/plvi_frontend.h): LineMatcher::SearchByProjection."""
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float), ("min_y", ctypes.c_float),
                ("max_y", ctypes.c_float), ("inv_w", ctypes.c_double), ("inv_h", ctypes.c_double),
                ("th", ctypes.c_float), ("angth", ctypes.c_float), ("grid_cols", ctypes.c_int),
                ("grid_rows", ctypes.c_int), ("range_hint", ctypes.c_int), ("nlevels", ctypes.c_int),
                ("scale_l", ctypes.c_float * 8)]


class FrustumCamera(ctypes.Structure):
    """plvi_frustum_camera (include/plvi_frontend.h): one camera of a frame for the frustum tests."""
    _fields_ = [("R", ctypes.c_float * 9), ("t", ctypes.c_float * 3), ("O", ctypes.c_float * 3),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("kb", ctypes.c_float * 4), ("model", ctypes.c_int)]


class FrustumParams(ctypes.Structure):
    """plvi_frustum_params (include/plvi_frontend.h): Frame::isInFrustum / isInFrustum_l of one frame."""
    _fields_ = [("cam", FrustumCamera * 2), ("two_camera", ctypes.c_int), ("mbf", ctypes.c_float),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float), ("min_y", ctypes.c_float),
                ("max_y", ctypes.c_float), ("view_cos_limit", ctypes.c_float), ("far_points", ctypes.c_int),
                ("far_th", ctypes.c_float), ("nlevels", ctypes.c_int), ("log_scale_factor", ctypes.c_float),
                ("level_ratio", ctypes.c_float * 16), ("compat", ctypes.c_uint)]


FRUSTUM_SEARCH, FRUSTUM_OBS, FRUSTUM_SEARCH_R, FRUSTUM_VISIBLE, FRUSTUM_TRACK = 1, 2, 4, 8, 16


def _same_len(n, **arrays):
    """The C entry points read n records from every host array: refuse a shorter (or longer) one
    instead of letting hipMemcpy read past its end."""
    for name, a in arrays.items():
        if a is not None and len(a) != n:
            raise ValueError(f"{name} has {len(a)} records, expected {n}")


def frustum_params_init(p):
    """plvi_frustum_params_init: PredictScale's level_ratio table from nlevels / log_scale_factor."""
    _check(load().plvi_frustum_params_init(ctypes.byref(p)), "plvi_frustum_params_init")
    return p


def frustum_points(params, pos, normal, dist, in_flags, proj=None, level=None, depth=None, proj_r=None,
                   level_r=None):
    """Frame::isInFrustum over one frame's local MapPoints (src/Frame.cc:758-847) from host memory.
    proj / level / depth (/ proj_r / level_r) are the MapPoint fields on entry (stale values are kept
    where the reference keeps them).  Returns (nToMatch, flags, proj, level, depth, proj_r, level_r)."""
    pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    n = len(pos)
    nr = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
    ds = np.ascontiguousarray(dist, np.float32).reshape(-1, 2)
    fi = np.ascontiguousarray(in_flags, np.uint8)
    pr = np.zeros((n, 4), np.float32) if proj is None else np.array(proj, np.float32).reshape(-1, 4)
    lv = np.zeros(n, np.int32) if level is None else np.array(level, np.int32)
    de = np.zeros(n, np.float32) if depth is None else np.array(depth, np.float32)
    two = bool(params.two_camera)
    prr = (np.zeros((n, 4), np.float32) if proj_r is None else np.array(proj_r, np.float32).reshape(-1, 4)) \
        if two else None
    lvr = (np.zeros(n, np.int32) if level_r is None else np.array(level_r, np.int32)) if two else None
    _same_len(n, normal=nr, dist=ds, in_flags=fi, proj=pr, level=lv, depth=de, proj_r=prr, level_r=lvr)
    fo = np.zeros(max(n, 1), np.uint8)
    nv = _check(load().plvi_frustum_points(ctypes.byref(params), _ptr(pos), _ptr(nr), _ptr(ds), _ptr(fi), n,
                                           _ptr(fo), _ptr(pr), _ptr(lv), None if prr is None else _ptr(prr),
                                           None if lvr is None else _ptr(lvr), _ptr(de)), "plvi_frustum_points")
    return nv, fo[:n], pr, lv, de, prr, lvr


def frustum_lines(params, sep, normal, dist, in_flags, desc=None, proj=None, angle=None):
    """Frame::isInFrustum_l over one frame's local MapLines (src/Frame.cc:849-933) from host memory.
    Returns (inview, proj, angle, compact, compact_desc): compact = mvpLocalMapLines_InFrustum as local
    indices, compact_desc = their descriptors (None without desc)."""
    sp = np.ascontiguousarray(sep, np.float64).reshape(-1, 6)
    n = len(sp)
    nr = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
    ds = np.ascontiguousarray(dist, np.float32).reshape(-1, 2)
    fi = np.ascontiguousarray(in_flags, np.uint8)
    de = None if desc is None else np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    pr = np.zeros((n, 4), np.float32) if proj is None else np.array(proj, np.float32).reshape(-1, 4)
    an = np.zeros(n, np.float64) if angle is None else np.array(angle, np.float64)
    _same_len(n, normal=nr, dist=ds, in_flags=fi, desc=de, proj=pr, angle=an)
    iv = np.zeros(max(n, 1), np.uint8)
    cp = np.zeros(max(n, 1), np.int32)
    cd = np.zeros((max(n, 1), 32), np.uint8)
    nc = _check(load().plvi_frustum_lines(ctypes.byref(params), _ptr(sp), _ptr(nr), _ptr(ds), _ptr(fi),
                                          None if de is None else _ptr(de), n, _ptr(iv), _ptr(pr), _ptr(an),
                                          _ptr(cp), _ptr(cd)), "plvi_frustum_lines")
    return iv[:n], pr, an, cp[:nc], (None if de is None else cd[:nc])


def grid_geometry(width, height):
    """Frame ctor grid geometry without distortion (mnMinX = 0, mnMaxX = cols, ...;
    Frame.cc:156-157): (min_x, max_x, min_y, max_y, inv_w, inv_h) as float32."""
    f = np.float32
    return (f(0), f(width), f(0), f(height), f(64) / (f(width) - f(0)), f(48) / (f(height) - f(0)))


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int),
                ("ini_th_fast", ctypes.c_int), ("min_th_fast", ctypes.c_int), ("compat", ctypes.c_uint)]


class LineParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("refine", ctypes.c_int), ("lsd_scale", ctypes.c_float),
                ("nlevels", ctypes.c_int), ("scale", ctypes.c_float), ("extractor", ctypes.c_int),
                ("compat", ctypes.c_uint)]


_lib = None
_runtime = None

c_int_p = ctypes.POINTER(ctypes.c_int)
c_void_pp = ctypes.POINTER(ctypes.c_void_p)


def _declare(lib):
    V, I, S, F, P = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_float, c_int_p
    sig = {
        "plvi_version": ([], ctypes.c_char_p),
        "plvi_device_count": ([], I),
        "plvi_orb_create": ([ctypes.POINTER(OrbParams), I, I, I, I, c_void_pp], I),
        "plvi_orb_destroy": ([V], I),
        "plvi_orb_extract": ([V, V, I, I, S, I, I, V, V, I, P, P], I),
        "plvi_orb_extract_batch": ([V, V, I, S, S, I, I, V], I),
        "plvi_orb_outputs": ([V, c_void_pp, c_void_pp, c_void_pp, c_void_pp, P], I),
        "plvi_orb_errors": ([V, V, P, V], I),
        "plvi_lines_errors": ([V, V, P, V], I),
        "plvi_lines_kernel_timing": ([V, I], I),
        "plvi_lines_kernel_timing_read": ([V, V, P], I),
        "plvi_lines_kernel_timing_read_kind": ([V, I, V, P], I),
        "plvi_line_match_nnr_inout": ([V, I, V, I, F, V, I], I),
        "plvi_line_match_inout": ([V, I, V, I, F, V, I], I),
        "plvi_orb_pyramid_level": ([V, I, I, V, P, P], I),
        "plvi_orb_pyramid_device": ([V, I, c_void_pp, ctypes.POINTER(S), P, P, P], I),
        "plvi_orb_scale_tables": ([V, V, V, V, V], I),
        "plvi_orb_level_quota": ([V, V], I),
        "plvi_orb_profile": ([V, I], I),
        "plvi_orb_profile_read": ([V, V, P], I),
        "plvi_orb_kernel_timing": ([V, I], I),
        "plvi_orb_kernel_timing_read": ([V, V, P], I),
        "plvi_orb_kernel_timing_read_kind": ([V, I, V, P], I),
        "plvi_orb_debug_node_cap": ([V, I], I),
        "plvi_hamming_knn2_batch": ([V, V, I, V, V, I, I, V, V, V, V, V], I),
        "plvi_hamming_knn2": ([V, I, V, I, V, V, V, V], I),
        "plvi_line_match_nnr": ([V, I, V, I, F, V], I),
        "plvi_line_match": ([V, I, V, I, F, V], I),
        "plvi_line_match_batch": ([V, V, I, V, V, I, I, F, V, V, V, V], I),
        "plvi_lines_create": ([ctypes.POINTER(LineParams), I, I, I, I, c_void_pp], I),
        "plvi_lines_destroy": ([V], I),
        "plvi_lines_extract": ([V, V, I, I, S, V, V, V, I, P], I),
        "plvi_lines_extract_batch": ([V, V, I, S, S, V], I),
        "plvi_lines_outputs": ([V, c_void_pp, c_void_pp, c_void_pp, c_void_pp, P], I),
        "plvi_lines_pyramid_level": ([V, I, I, V, P, P], I),
        "plvi_lines_scale_tables": ([V, V, V, V, V], I),
        "plvi_lines_profile": ([V, I], I),
        "plvi_lines_profile_read": ([V, V, P], I),
        "plvi_lines_debug_stats": ([V, V], I),
        "plvi_lines_debug_mw_stats": ([V, V], I),
        "plvi_lines_debug_planes": ([V, I, I, V, V, V, P, P], I),
        "plvi_lines_debug_sobel": ([V, I, I, V, P, P], I),
        "plvi_descriptor_distance_batch": ([V, V, I, I, V, V], I),
        "plvi_search_by_bow": ([F, I, V, V, V, I, V, V, I, V, V, V, I, V, V, I, V, V], I),
        "plvi_search_by_bow_stereo": ([F, I, V, V, V, I, V, V, I, V, V, V, I, V, V, I, V, I, V], I),
        "plvi_search_by_bow_stereo_batch": ([I, F, I, I, I, I, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V,
                                             V], I),
        "plvi_search_by_bow_batch": ([I, F, I, I, I, I, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V, V], I),
        "plvi_line_match_grid": ([V, V, I, I, I, V, V, V, V, I, I, I, I, I, I, V], I),
        "plvi_line_match_grid_batch": ([I, V, V, V, I, I, I, V, V, I, V, V, V, I, I, I, I, I, I, V, V, V, V], I),
        "plvi_frame_extract_batch": ([V, V, V, I, S, S, I, I, V], I),
        "plvi_assign_grid_batch": ([V, V, I, I, V, V, V, V], I),
        "plvi_undistort_points": ([V, V, I, V, V], I),
        "plvi_undistort_keypoints_batch": ([V, V, V, I, I, V, V], I),
        "plvi_undistort_keylines_batch": ([V, V, V, I, I, V, V], I),
        "plvi_image_bounds": ([V, I, I, V], I),
        "plvi_search_by_projection_batch": ([I, V, V, V, V, I, V, V, V, V, V, V, V, V, V, V, I, V, V, V], I),
        "plvi_search_by_projection": ([V, V, V, I, V, V, V, V, V, V, V, I, V], I),
        "plvi_stereo_frame_extract_batch": ([V, V, V, V, V, V, I, S, S, I, I, V], I),
        "plvi_event_create": ([c_void_pp], I),
        "plvi_event_record": ([V, V], I),
        "plvi_stream_wait_event": ([V, V], I),
        "plvi_event_destroy": ([V], I),
        "plvi_frame_orb_event": ([V, c_void_pp], I),
        "plvi_frame_extract_match_batch": ([V, V, V, I, S, S, I, I, V, V, V, V, F, V, V, V, V], I),
        "plvi_stream_create": ([c_void_pp], I),
        "plvi_stream_destroy": ([V], I),
        "plvi_stream_synchronize": ([V], I),
        "plvi_search_for_initialization_batch": ([I, V, V, V, V, I, V, V, V, V, I, V, V, V, V, V], I),
        "plvi_line_search_init_batch": ([V, V, I, V, V, I, I, V, V, V, V, V], I),
        "plvi_search_local_batch": ([I, V, V, V, V, I, V, V, V, V, V, V, V, V, V, I, V, V, V], I),
        "plvi_search_local": ([V, V, V, I, V, V, V, V, V, V, I, V], I),
        "plvi_search_by_projection_stereo_batch": ([I, V, V, V, V, V, I, V, V, V, V, V, V, I, V, V, V, V, V, V, V, V,
                                                    V, V, I, V, V, V, V], I),
        "plvi_search_by_projection_stereo": ([V, V, V, V, I, V, V, V, I, V, V, V, V, V, V, V, I, V, V], I),
        "plvi_search_local_stereo_batch": ([I, V, V, V, V, I, V, V, V, V, V, V, V, I, V, V, V, V, V, V, V, V, V, V,
                                            V, I, V, V, V, V], I),
        "plvi_search_local_stereo": ([V, V, V, I, V, V, V, V, I, V, V, V, V, V, V, V, V, I, V, V], I),
        "plvi_search_reloc_batch": ([I, V, V, V, V, I, V, V, V, V, V, V, V, V, V, V, I, V, V, V], I),
        "plvi_search_reloc": ([V, V, V, I, V, V, V, V, V, V, V, I, V], I),
        "plvi_line_search_projection_batch": ([I, V, V, V, V, V, I, V, V, I, V, V, V, V, V, I, V, V, V, V], I),
        "plvi_line_search_projection": ([V, V, V, V, I, V, V, V, V, V, V, I, V], I),
        "plvi_vocab_load_text": ([ctypes.c_char_p, I, I, c_void_pp], I),
        "plvi_vocab_create": ([I, I, I, I, I, V, V, V, V, I, c_void_pp], I),
        "plvi_vocab_destroy": ([V], I),
        "plvi_vocab_info": ([V, V], I),
        "plvi_vocab_transform": ([V, V, I, I, V, V, P, V, V, V, P], I),
        "plvi_vocab_transform_features": ([V, V, I, I, V, V], I),
        "plvi_vocab_transform_batch": ([V, V, V, I, I, I, V, V, V, V, V, V, V, V, V, V], I),
        "plvi_stereo_match_batch": ([V, V, I, F, F, V, V, V, V, V], I),
        "plvi_stereo_match": ([V, V, I, V, V, I, I, V, V, V, V, V, V, V, F, F, V, V], I),
        "plvi_stereo_lines_scratch_bytes": ([I, I, I, I], S),
        "plvi_stereo_lines_batch": ([I, V, V, V, I, V, V, V, I, V, I, I, F, I, I, V, S, V, V, V, V, V, V, V], I),
        "plvi_stereo_lines": ([V, V, I, V, V, I, V, I, I, F, I, V, V, V, V], I),
        "plvi_frustum_params_init": ([V], I),
        "plvi_frustum_points_batch": ([I, V, V, V, V, V, V, I, V, V, V, V, V, V, V, V], I),
        "plvi_frustum_points": ([V, V, V, V, V, I, V, V, V, V, V, V], I),
        "plvi_frustum_lines_batch": ([I, V, V, V, V, V, V, V, I, V, V, V, V, V, V, V], I),
        "plvi_frustum_lines": ([V, V, V, V, V, V, I, V, V, V, V, V], I),
        "plvi_local_lines_filter_batch": ([I, V, V, V, V, I, V, V, V, V, I, V, V, V, V], I),
        "plvi_device_malloc": ([c_void_pp, S], I),
        "plvi_device_free": ([V], I),
        "plvi_memcpy": ([V, V, S, I], I),
        "plvi_memcpy_async": ([V, V, S, I, V], I),
        "plvi_device_synchronize": ([], I),
        "plvi_graph_capture_begin": ([V], I),
        "plvi_graph_capture_end": ([V, c_void_pp], I),
        "plvi_graph_launch": ([V, V], I),
        "plvi_graph_destroy": ([V], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def load(runtime=None):
    """Load the HIP library (raises if it was not built: there is no fallback).

    Which HIP runtime the library binds to is decided here, once per process:
    PyTorch's bundled libamdhip64 (HIP 7.0 on this image) and /opt/rocm's
    (7.2) share the SONAME libamdhip64.so.7, so whichever loads first serves
    both -- unless ours comes first and torch is imported later, in which case
    torch loads its own copy by file name and that second runtime finds no
    device.  `runtime`:

    * "torch": import torch first (one runtime for both).  On the 7.0 runtime
      `plvi_frame_extract_batch` / `plvi_stereo_frame_extract_batch` refuse
      stream capture with PLVI_E_CAPTURE; everything else
      behaves identically.
    * "system": do not import torch; the library binds to /opt/rocm's runtime
      (capture supported).  Do not import torch later in the same process.
    * None (default): "torch" if torch is already imported, else the
      PLVI_RUNTIME environment variable ("torch" / "system"; PLVI_NO_TORCH=1
      means "system"), else "torch" when torch is installed -- the safe choice
      for a process that may import torch later.
    """
    global _lib, _runtime
    if _lib is None:
        if runtime is None:
            if "torch" in sys.modules:
                runtime = "torch"
            elif os.environ.get("PLVI_NO_TORCH"):
                runtime = "system"
            else:
                runtime = os.environ.get("PLVI_RUNTIME", "torch")
        if runtime not in ("torch", "system"):
            raise ValueError(f"plvi.load: runtime must be 'torch' or 'system', not {runtime!r}")
        if runtime == "torch":
            try:
                import torch  # noqa: F401
            except ImportError:
                runtime = "system"
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C pl-vi-orbslam3_amd`")
        _lib = _declare(ctypes.CDLL(str(LIB_PATH)))
        _runtime = runtime
    elif runtime is not None and runtime != _runtime:
        raise RuntimeError(f"plvi.load: library already bound to the {_runtime!r} HIP runtime")
    return _lib


def bound_runtime():
    """'torch' or 'system': the HIP runtime the loaded library is bound to (None before load())."""
    return _runtime


def exported_symbols():
    """Function names declared in include/plvi_frontend.h."""
    import re
    txt = HEADER_PATH.read_text()
    return sorted(set(re.findall(r"\b(plvi_[a-z0-9_]+)\s*\(", txt)))


class DeviceBuffer:
    """hipMalloc'd buffer owned from Python (no torch needed)."""

    def __init__(self, nbytes):
        self._lib = load()
        p = ctypes.c_void_p()
        _check(self._lib.plvi_device_malloc(ctypes.byref(p), max(1, nbytes)), "plvi_device_malloc")
        self.ptr, self.nbytes = p.value, nbytes

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(self._lib.plvi_memcpy(ctypes.c_void_p(self.ptr), _ptr(arr), arr.nbytes, 1), "plvi_memcpy")

    def download(self, arr, src_ptr=None):
        _check(self._lib.plvi_memcpy(_ptr(arr), ctypes.c_void_p(src_ptr or self.ptr), arr.nbytes, 2),
               "plvi_memcpy")
        return arr

    def __del__(self):
        try:
            if self.ptr:
                self._lib.plvi_device_free(ctypes.c_void_p(self.ptr))
                self.ptr = None
        except Exception:
            pass


def download(ptr, arr):
    """Copy device memory at `ptr` into numpy array `arr` (synchronous)."""
    _check(load().plvi_memcpy(_ptr(arr), ctypes.c_void_p(ptr), arr.nbytes, 2), "plvi_memcpy")
    return arr


def _check(rc, what):
    if rc < 0:
        raise PlviError(rc, what)
    return rc


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class ORBextractor:
    """ORB_SLAM3::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST).

    ``extractor(image, mask, vLappingArea)`` returns ``(monoIndex, keypoints,
    descriptors)`` like operator() (src/ORBextractor.cc:1068): keypoints is a
    structured array in cv::KeyPoint layout, descriptors an N x 32 uint8 array.
    An empty image returns ``(-1, empty, empty)``.
    """

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, width=640, height=480,
                 max_batch=1, device=0, compat=0):
        self._lib = load()
        self.params = OrbParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, compat)
        self.width, self.height, self.max_batch = width, height, max_batch
        self.nlevels = nlevels
        h = ctypes.c_void_p()
        _check(self._lib.plvi_orb_create(ctypes.byref(self.params), width, height, max_batch, device,
                                         ctypes.byref(h)), "plvi_orb_create")
        self._h = h
        cap = ctypes.c_int()
        self._lib.plvi_orb_outputs(self._h, None, None, None, None, ctypes.byref(cap))
        self.kp_cap = cap.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.plvi_orb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __call__(self, image, mask=None, vLappingArea=(0, 0)):
        """operator(): any frame size (a new size re-plans the handle); an
        empty image returns (-1, empty, empty) from the C-ABI's PLVI_E_EMPTY."""
        image = np.ascontiguousarray(image if image is not None else np.zeros((0, 0)), dtype=np.uint8)
        h, w = image.shape if image.ndim == 2 else (0, 0)
        if (w, h) != (self.width, self.height) and w > 0 and h > 0:
            self.width, self.height = w, h
        kps = np.zeros(self.kp_cap, KEYPOINT_DTYPE)
        desc = np.zeros((self.kp_cap, 32), np.uint8)
        n, mono = ctypes.c_int(), ctypes.c_int()
        rc = self._lib.plvi_orb_extract(self._h, _ptr(image) if image.size else None, w, h, w,
                                        int(vLappingArea[0]), int(vLappingArea[1]), _ptr(kps), _ptr(desc),
                                        self.kp_cap, ctypes.byref(n), ctypes.byref(mono))
        if rc == PLVI_E_EMPTY:
            return -1, np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8)
        if rc == PLVI_E_CAPACITY:  # a re-planned (larger) frame: grow the host buffers once
            self._refresh_cap()
            return self(image, mask, vLappingArea)
        _check(rc, "plvi_orb_extract")
        self._refresh_cap()
        return mono.value, kps[:n.value].copy(), desc[:n.value].copy()

    def _refresh_cap(self):
        cap = ctypes.c_int()
        self._lib.plvi_orb_outputs(self._h, None, None, None, None, ctypes.byref(cap))
        self.kp_cap = cap.value

    def errors(self, stream=None, per_frame=False):
        """Read-and-clear device error flags of the batches run so far (PLVI_FERR_*)."""
        flags = np.zeros(self.max_batch, np.int32)
        anyf = ctypes.c_int()
        _check(self._lib.plvi_orb_errors(self._h, _ptr(flags), ctypes.byref(anyf), ctypes.c_void_p(stream or 0)),
               "plvi_orb_errors")
        return flags if per_frame else anyf.value

    # --- batched device path (bench / multi-frame) ---------------------------
    def extract_batch(self, d_frames_ptr, n_frames, frame_stride, row_stride, lap=(0, 0), stream=None):
        _check(self._lib.plvi_orb_extract_batch(self._h, ctypes.c_void_p(d_frames_ptr), n_frames, frame_stride,
                                                row_stride, lap[0], lap[1], ctypes.c_void_p(stream or 0)),
               "plvi_orb_extract_batch")

    def outputs(self):
        """Device pointers (kps, desc, count, mono) and per-frame capacity."""
        kp, de, co, mo = (ctypes.c_void_p() for _ in range(4))
        cap = ctypes.c_int()
        _check(self._lib.plvi_orb_outputs(self._h, ctypes.byref(kp), ctypes.byref(de), ctypes.byref(co),
                                          ctypes.byref(mo), ctypes.byref(cap)), "plvi_orb_outputs")
        return kp.value, de.value, co.value, mo.value, cap.value

    ORB_STAGES = ("level", "nms", "sat", "octree", "best", "describe", "assemble")

    def profile(self, enable=True):
        _check(self._lib.plvi_orb_profile(self._h, int(enable)), "plvi_orb_profile")

    def profile_read(self):
        ms = np.zeros(7, np.float32)
        runs = ctypes.c_int()
        _check(self._lib.plvi_orb_profile_read(self._h, _ptr(ms), ctypes.byref(runs)), "plvi_orb_profile_read")
        return dict(zip(self.ORB_STAGES, ms.tolist())), runs.value

    def kernel_timing(self, enable=True):
        """Event pair around every blur + FAST and pyramid kernel launch (rooflines)."""
        _check(self._lib.plvi_orb_kernel_timing(self._h, int(enable)), "plvi_orb_kernel_timing")

    def kernel_timing_read(self, kind=0):
        """(total ms, launches) since kernel_timing(True): kind 0 = orb_blur_fast_kernel, 1 = orb_pyramid_kernel."""
        tot = ctypes.c_float()
        n = ctypes.c_int()
        _check(self._lib.plvi_orb_kernel_timing_read_kind(self._h, int(kind), ctypes.byref(tot), ctypes.byref(n)),
               "plvi_orb_kernel_timing_read_kind")
        return tot.value, n.value

    # --- reference getters ---------------------------------------------------
    def _tables(self):
        out = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        _check(self._lib.plvi_orb_scale_tables(self._h, *[_ptr(a) for a in out]), "plvi_orb_scale_tables")
        return out

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(np.float32(self.params.scale_factor))

    def GetScaleFactors(self):
        return self._tables()[0]

    def GetInverseScaleFactors(self):
        return self._tables()[1]

    def GetScaleSigmaSquares(self):
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._tables()[3]

    def level_quota(self):
        q = np.zeros(self.nlevels, np.int32)
        _check(self._lib.plvi_orb_level_quota(self._h, _ptr(q)), "plvi_orb_level_quota")
        return q

    def pyramid_level(self, level, frame=0):
        """mvImagePyramid[level] of the last call (lazy D2H)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_orb_pyramid_level(self._h, frame, level, None, ctypes.byref(w), ctypes.byref(h)),
               "plvi_orb_pyramid_level")
        out = np.zeros((h.value, w.value), np.uint8)
        _check(self._lib.plvi_orb_pyramid_level(self._h, frame, level, _ptr(out), None, None),
               "plvi_orb_pyramid_level")
        return out

    @property
    def mvImagePyramid(self):
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def pyramid_device(self, level):
        """Device view of mvImagePyramid[level]: (frame-0 pointer, frame stride, w, h)."""
        p, fs = ctypes.c_void_p(), ctypes.c_size_t()
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_orb_pyramid_device(self._h, level, ctypes.byref(p), ctypes.byref(fs), ctypes.byref(w),
                                                 ctypes.byref(h), None), "plvi_orb_pyramid_device")
        return p.value, fs.value, w.value, h.value


class Lineextractor:
    """ORB_SLAM3::Lineextractor(lsd_nfeatures, lsd_refine, lsd_scale, nlevels, scale, extractor).

    ``extractor(image, mask)`` returns ``(keylines, descriptors, keylineFunctions)``
    as operator() fills them (src/LineExtractor.cc:45-117): keylines in KeyLine
    layout, n x 32 LBD descriptors, n x 3 normalised line equations.
    """

    STAGES = ("pyramid", "lsd_prep", "region_grow", "assemble", "lbd")

    def __init__(self, lsd_nfeatures, lsd_refine, lsd_scale, nlevels, scale, extractor=0, width=640, height=480,
                 max_batch=1, device=0, compat=0):
        self._lib = load()
        self.params = LineParams(lsd_nfeatures, lsd_refine, lsd_scale, nlevels, scale, extractor, compat)
        self.width, self.height, self.max_batch, self.nlevels = width, height, max_batch, nlevels
        h = ctypes.c_void_p()
        _check(self._lib.plvi_lines_create(ctypes.byref(self.params), width, height, max_batch, device,
                                           ctypes.byref(h)), "plvi_lines_create")
        self._h = h
        cap = ctypes.c_int()
        self._lib.plvi_lines_outputs(self._h, None, None, None, None, ctypes.byref(cap))
        self.cap = cap.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.plvi_lines_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __call__(self, image, mask=None):
        image = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = image.shape
        kl = np.zeros(self.cap, KEYLINE_DTYPE)
        desc = np.zeros((self.cap, 32), np.uint8)
        fn = np.zeros((self.cap, 3), np.float64)
        n = ctypes.c_int()
        _check(self._lib.plvi_lines_extract(self._h, _ptr(image), w, h, w, _ptr(kl), _ptr(desc), _ptr(fn), self.cap,
                                            ctypes.byref(n)), "plvi_lines_extract")
        self.width, self.height = w, h
        k = n.value
        return kl[:k].copy(), desc[:k].copy(), fn[:k].copy()

    def errors(self, stream=None, per_frame=False):
        """Read-and-clear device error flags of the batches run so far (PLVI_FERR_*)."""
        flags = np.zeros(self.max_batch, np.int32)
        anyf = ctypes.c_int()
        _check(self._lib.plvi_lines_errors(self._h, _ptr(flags), ctypes.byref(anyf), ctypes.c_void_p(stream or 0)),
               "plvi_lines_errors")
        return flags if per_frame else anyf.value

    def extract_batch(self, d_frames_ptr, n_frames, frame_stride, row_stride, stream=None):
        _check(self._lib.plvi_lines_extract_batch(self._h, ctypes.c_void_p(d_frames_ptr), n_frames, frame_stride,
                                                  row_stride, ctypes.c_void_p(stream or 0)),
               "plvi_lines_extract_batch")

    def outputs(self):
        kl, de, fn, co = (ctypes.c_void_p() for _ in range(4))
        cap = ctypes.c_int()
        _check(self._lib.plvi_lines_outputs(self._h, ctypes.byref(kl), ctypes.byref(de), ctypes.byref(fn),
                                            ctypes.byref(co), ctypes.byref(cap)), "plvi_lines_outputs")
        return kl.value, de.value, fn.value, co.value, cap.value

    def profile(self, enable=True):
        _check(self._lib.plvi_lines_profile(self._h, int(enable)), "plvi_lines_profile")

    def profile_read(self):
        ms = np.zeros(5, np.float32)
        runs = ctypes.c_int()
        _check(self._lib.plvi_lines_profile_read(self._h, _ptr(ms), ctypes.byref(runs)), "plvi_lines_profile_read")
        return dict(zip(self.STAGES, ms.tolist())), runs.value

    def kernel_timing(self, enable=True):
        """Event pair around every lsd_prep_kernel and LBD Gaussian + Sobel launch (rooflines)."""
        _check(self._lib.plvi_lines_kernel_timing(self._h, int(enable)), "plvi_lines_kernel_timing")

    def kernel_timing_read(self, kind=0):
        """(total ms, launches) since kernel_timing(True): kind 0 = lsd_prep_kernel, 1 = lbd_sobel0_kernel,
        2 = lbd_sobel1_kernel."""
        tot = ctypes.c_float()
        n = ctypes.c_int()
        _check(self._lib.plvi_lines_kernel_timing_read_kind(self._h, int(kind), ctypes.byref(tot), ctypes.byref(n)),
               "plvi_lines_kernel_timing_read_kind")
        return tot.value, n.value

    def pyramid_level(self, level, frame=0):
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_lines_pyramid_level(self._h, frame, level, None, ctypes.byref(w), ctypes.byref(h)),
               "plvi_lines_pyramid_level")
        out = np.zeros((h.value, w.value), np.uint8)
        _check(self._lib.plvi_lines_pyramid_level(self._h, frame, level, _ptr(out), None, None),
               "plvi_lines_pyramid_level")
        return out

    def debug_planes(self, level, frame=0):
        """(deg f32, modgrad f64, cos/sin f32 [h, w, 2]) LSD planes of the last batch (diagnostic)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_lines_debug_planes(self._h, frame, level, None, None, None, ctypes.byref(w),
                                                  ctypes.byref(h)), "plvi_lines_debug_planes")
        deg = np.zeros((h.value, w.value), np.float32)
        mg = np.zeros((h.value, w.value), np.float64)
        cs = np.zeros((h.value, w.value, 2), np.float32)
        _check(self._lib.plvi_lines_debug_planes(self._h, frame, level, _ptr(deg), _ptr(mg), _ptr(cs), None, None),
               "plvi_lines_debug_planes")
        return deg, mg, cs

    def debug_sobel(self, level, frame=0):
        """(dx, dy) int16 LBD Sobel planes of the last batch (diagnostic)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_lines_debug_sobel(self._h, frame, level, None, ctypes.byref(w), ctypes.byref(h)),
               "plvi_lines_debug_sobel")
        g = np.zeros((h.value, w.value, 2), np.int16)
        _check(self._lib.plvi_lines_debug_sobel(self._h, frame, level, _ptr(g), None, None), "plvi_lines_debug_sobel")
        return g[..., 0].copy(), g[..., 1].copy()

    def scale_tables(self):
        out = [np.zeros(self.nlevels, np.float32) for _ in range(4)]
        _check(self._lib.plvi_lines_scale_tables(self._h, *[_ptr(a) for a in out]), "plvi_lines_scale_tables")
        return out


def hamming_knn2(q, t):
    """BFMatcher(NORM_HAMMING).knnMatch(q, t, 2) -> (idx0, d0, idx1, d1) arrays."""
    lib = load()
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    nq, nt = q.shape[0], t.shape[0]
    out = [np.zeros(nq, np.int32) for _ in range(4)]
    _check(lib.plvi_hamming_knn2(_ptr(q), nq, _ptr(t), nt, *[_ptr(o) for o in out]), "plvi_hamming_knn2")
    return tuple(out)


def grid_csr(grid):
    """GridStructure (grid[x][y] = list of indices) -> (cols, rows, cell_off, cell_idx)."""
    cols, rows = len(grid), len(grid[0])
    off = np.zeros(cols * rows + 1, np.int32)
    idx = []
    for x in range(cols):
        for y in range(rows):
            idx.extend(grid[x][y])
            off[x * rows + y + 1] = len(idx)
    return cols, rows, off, np.array(idx if idx else [0], np.int32)


class LineMatcher:
    """ORB_SLAM3::LineMatcher static Hamming matchers (src/LineMatcher.cpp)."""

    @staticmethod
    def _inout(fn, name, desc1, desc2, nnr, matches_12):
        d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
        prev = np.zeros(0, np.int32) if matches_12 is None else np.ascontiguousarray(matches_12, np.int32)
        m = np.full(max(d1.shape[0], prev.size, 1), -1, np.int32)
        m[:prev.size] = prev
        n = _check(fn(_ptr(d1), d1.shape[0], _ptr(d2), d2.shape[0], nnr, _ptr(m), prev.size), name)
        return n, m[:d1.shape[0]].copy()

    @staticmethod
    def matchNNR(desc1, desc2, nnr, matches_12=None):
        """LineMatcher::matchNNR (LineMatcher.cpp:41-61).  matches_12: the caller's
        existing vector (kept through resize(rows, -1) like the reference), or None."""
        lib = load()
        return LineMatcher._inout(lib.plvi_line_match_nnr_inout, "plvi_line_match_nnr_inout", desc1, desc2, nnr,
                                  matches_12)

    @staticmethod
    def match(desc1, desc2, nnr, matches_12=None):
        """LineMatcher::match(desc1, desc2, nnr, matches_12) (LineMatcher.cpp:92-111)."""
        lib = load()
        return LineMatcher._inout(lib.plvi_line_match_inout, "plvi_line_match_inout", desc1, desc2, nnr, matches_12)

    @staticmethod
    def SearchByProjection(params, cur_angle, cur_desc, grid, last_flags, last_x3dc, last_octave, ml_desc,
                           cur_blocked=None):
        """LineMatcher::SearchByProjection(CurrentFrame, LastFrame, grid, th, angth) (src/LineMatcher.cpp:274-372).
        params: LineProjParams; grid: grid[x][y] lists of current-line indices (grid_Line); last_x3dc: n x 6
        camera-frame endpoints.  Returns (count, match) with match[i2] = last-frame line index or -1."""
        lib = load()
        ca = np.ascontiguousarray(cur_angle, np.float32)
        cd = np.ascontiguousarray(cur_desc, np.uint8).reshape(-1, 32)
        cols, rows, off, idx = grid_csr(grid)
        params.grid_cols, params.grid_rows = cols, rows
        fl = np.ascontiguousarray(last_flags, np.uint8)
        x3 = np.ascontiguousarray(last_x3dc, np.float32).reshape(-1, 6)
        oc = np.ascontiguousarray(last_octave, np.int32)
        md = np.ascontiguousarray(ml_desc, np.uint8).reshape(-1, 32)
        cb = None if cur_blocked is None else np.ascontiguousarray(cur_blocked, np.uint8)
        out = np.full(max(len(ca), 1), -1, np.int32)
        n = _check(lib.plvi_line_search_projection(ctypes.byref(params), _ptr(ca), _ptr(cd),
                                                   None if cb is None else _ptr(cb), len(ca), _ptr(off), _ptr(idx),
                                                   _ptr(fl), _ptr(x3), _ptr(oc), _ptr(md), len(fl), _ptr(out)),
                   "plvi_line_search_projection")
        return n, out[:len(ca)]

    @staticmethod
    def matchGrid(lines1, desc1, grid, desc2, directions2, window=((7, 0), (2, 2)), range_hint=1):
        """LineMatcher::matchGrid (src/LineMatcher.cpp:191-272).  lines1: n1 x 4 ints (line_2d grid coords),
        grid: grid[x][y] lists of right-line indices, directions2: n2 x 2.  range_hint: 1 = libstdc++ <= GCC 10
        candidate order (the reference's toolchain), 0 = GCC >= 11.  Returns (nmatches, matches_12)."""
        lib = load()
        l1 = np.ascontiguousarray(lines1, np.int32).reshape(-1, 4)
        d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
        v2 = np.ascontiguousarray(directions2, np.float64).reshape(-1, 2)
        cols, rows, off, idx = grid_csr(grid)
        m = np.full(max(len(l1), 1), -1, np.int32)
        (w0, w1), (h0, h1) = window
        n = _check(lib.plvi_line_match_grid(_ptr(l1), _ptr(d1), len(l1), cols, rows, _ptr(off), _ptr(idx), _ptr(d2),
                                            _ptr(v2), len(d2), w0, w1, h0, h1, int(range_hint), _ptr(m)),
                   "plvi_line_match_grid")
        return n, m[:len(l1)]


def feature_vector_csr(fv):
    """DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as given by a
    dict {node_id: [keypoint indices]} -> (node ids ascending, offsets, indices)."""
    nodes = np.array(sorted(fv), dtype=np.int32)
    off = np.zeros(len(nodes) + 1, np.int32)
    idx = []
    for i, n in enumerate(nodes):
        idx.extend(fv[int(n)])
        off[i + 1] = len(idx)
    return nodes, off, np.array(idx, dtype=np.int32)


class ORBmatcher:
    """ORB_SLAM3::ORBmatcher(nnratio=0.6, checkOri=true) (include/ORBmatcher.h:39-68)."""

    def __init__(self, nnratio=0.6, checkOri=True):
        self._lib = load()
        self.nnratio = float(nnratio)
        self.check_orientation = bool(checkOri)

    def SearchByBoW(self, kf_desc, kf_angle, kf_live, kf_featvec, f_desc, f_angle, f_featvec, f_nleft=-1):
        """SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:269-471); f_nleft = F.Nleft
        (-1: one camera; else the two-camera branch, :321-420).  Returns (nmatches, match_kf) with
        match_kf[iF] = KF keypoint index or -1."""
        kd = np.ascontiguousarray(kf_desc, np.uint8)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        kl = np.ascontiguousarray(kf_live, np.uint8)
        fd = np.ascontiguousarray(f_desc, np.uint8)
        fa = np.ascontiguousarray(f_angle, np.float32)
        kn, ko, ki = feature_vector_csr(kf_featvec)
        fn, fo, fi = feature_vector_csr(f_featvec)
        out = np.full(max(len(fd), 1), -1, np.int32)
        n = _check(self._lib.plvi_search_by_bow_stereo(self.nnratio, int(self.check_orientation), _ptr(kd),
                                                       _ptr(ka), _ptr(kl), len(kd), _ptr(kn), _ptr(ko), len(kn),
                                                       _ptr(ki), _ptr(fd), _ptr(fa), len(fd), _ptr(fn), _ptr(fo),
                                                       len(fn), _ptr(fi), int(f_nleft), _ptr(out)),
                   "plvi_search_by_bow_stereo")
        return n, out[:len(fd)]

    def SearchByProjection(self, params, cur_kps, cur_desc, last_x3dc, last_octave, last_angle, mp_desc,
                           last_flags, cur_blocked=None, cur_uright=None):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono) (src/ORBmatcher.cc:1962-2178) with
        mbCheckOrientation = checkOri of this matcher.  params: ProjParams (th, camera, grid, bounds,
        scale factors); cur_kps: mvKeysUn (KEYPOINT_DTYPE); last_*: see include/plvi_frontend.h.
        Returns (nmatches, match) with match[i2] = LastFrame index, -2 (nulled) or -1 (untouched)."""
        params.check_orientation = int(self.check_orientation)
        ck = np.ascontiguousarray(cur_kps).view(KEYPOINT_DTYPE)
        cd = np.ascontiguousarray(cur_desc, np.uint8).reshape(-1, 32)
        n = len(ck)
        x3 = np.ascontiguousarray(last_x3dc, np.float32).reshape(-1, 3)
        lo = np.ascontiguousarray(last_octave, np.int32)
        la = np.ascontiguousarray(last_angle, np.float32)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        lf = np.ascontiguousarray(last_flags, np.uint8)
        cb = None if cur_blocked is None else np.ascontiguousarray(cur_blocked, np.uint8)
        cu = None if cur_uright is None else np.ascontiguousarray(cur_uright, np.float32)
        out = np.full(max(n, 1), -1, np.int32)
        nm = _check(self._lib.plvi_search_by_projection(ctypes.byref(params), _ptr(ck), _ptr(cd), n,
                                                        None if cb is None else _ptr(cb),
                                                        None if cu is None else _ptr(cu), _ptr(x3), _ptr(lo),
                                                        _ptr(la), _ptr(md), _ptr(lf), len(lf), _ptr(out)),
                    "plvi_search_by_projection")
        return nm, out[:n]

    def SearchByProjectionLocal(self, params, kps, desc, mp_flags, mp_proj, mp_level, mp_desc, blocked=None,
                                uright=None):
        """SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
        (src/ORBmatcher.cc:44-145, monocular / rectified branch) with this matcher's nnratio.  params:
        LocalParams (grid, th, scale factors); kps: F.mvKeysUn; mp_*: per MapPoint (vector order) flags (bit0
        searched, bit1 Observations() > 0), proj (n x 4: mTrackProjX, mTrackProjY, mTrackProjXR,
        mTrackViewCos), mnTrackScaleLevel, descriptor.  Returns (nmatches, match) with match[idx] = MapPoint
        index stored in F.mvpMapPoints[idx] or -1."""
        params.nnratio = self.nnratio
        k = np.ascontiguousarray(kps).view(KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        fl = np.ascontiguousarray(mp_flags, np.uint8)
        pr = np.ascontiguousarray(mp_proj, np.float32).reshape(-1, 4)
        lv = np.ascontiguousarray(mp_level, np.int32)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        cb = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        cu = None if uright is None else np.ascontiguousarray(uright, np.float32)
        out = np.full(max(len(k), 1), -1, np.int32)
        nm = _check(self._lib.plvi_search_local(ctypes.byref(params), _ptr(k), _ptr(d), len(k),
                                                None if cb is None else _ptr(cb), None if cu is None else _ptr(cu),
                                                _ptr(fl), _ptr(pr), _ptr(lv), _ptr(md), len(fl), _ptr(out)),
                    "plvi_search_local")
        return nm, out[:len(k)]

    def SearchByProjectionStereo(self, params, kps, desc, kps_r, desc_r, x3dc, x3dr, last_octave, last_angle,
                                 mp_desc, last_flags, kb8=None, blocked=None, blocked_r=None):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono) with a two-camera CurrentFrame
        (CurrentFrame.Nleft != -1, src/ORBmatcher.cc:1985-2175), rotation check = checkOri of this matcher.
        params: ProjParams (camera fx/fy/cx/cy, bounds, grid, th, forward / backward, scale factors); kb8:
        KannalaBrandt8 k1..k4 (None = Pinhole); kps / desc: mvKeys and descriptor rows 0..Nleft-1; kps_r /
        desc_r: mvKeysRight and rows Nleft..; per LastFrame point: x3Dc, x3Dr = mTrl * x3Dc, octave, angle,
        descriptor, flags (bit0 MapPoint and not an outlier, bit1 Observations() > 0).  Returns (nmatches,
        match, match_r) with -2 = set to NULL by the rotation filter."""
        params.check_orientation = int(self.check_orientation)
        k = np.ascontiguousarray(kps).view(KEYPOINT_DTYPE)
        kr = np.ascontiguousarray(kps_r).view(KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        dr = np.ascontiguousarray(desc_r, np.uint8).reshape(-1, 32)
        x3 = np.ascontiguousarray(x3dc, np.float32).reshape(-1, 3)
        x3r = np.ascontiguousarray(x3dr, np.float32).reshape(-1, 3)
        lo = np.ascontiguousarray(last_octave, np.int32)
        la = np.ascontiguousarray(last_angle, np.float32)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        lf = np.ascontiguousarray(last_flags, np.uint8)
        opt = lambda a, t: None if a is None else np.ascontiguousarray(a, t)  # noqa: E731
        kb, cb, cbr = opt(kb8, np.float32), opt(blocked, np.uint8), opt(blocked_r, np.uint8)
        pp = lambda a: None if a is None else _ptr(a)  # noqa: E731
        out = np.full(max(len(k), 1), -1, np.int32)
        outr = np.full(max(len(kr), 1), -1, np.int32)
        nm = _check(self._lib.plvi_search_by_projection_stereo(
            ctypes.byref(params), pp(kb), _ptr(k), _ptr(d), len(k), pp(cb), _ptr(kr), _ptr(dr), len(kr), pp(cbr),
            _ptr(x3), _ptr(x3r), _ptr(lo), _ptr(la), _ptr(md), _ptr(lf), len(lf), _ptr(out), _ptr(outr)),
            "plvi_search_by_projection_stereo")
        return nm, out[:len(k)], outr[:len(kr)]

    def SearchByProjectionLocalStereo(self, params, kps, desc, kps_r, desc_r, mp_flags, mp_proj, mp_level,
                                      mp_proj_r, mp_level_r, mp_desc, blocked=None, blocked_r=None, l2r=None,
                                      r2l=None):
        """SearchByProjection(Frame&, const vector<MapPoint*>&, ...) on a two-camera Frame (F.Nleft != -1,
        src/ORBmatcher.cc:44-214).  kps / desc: mvKeys and descriptor rows 0..Nleft-1; kps_r / desc_r:
        mvKeysRight and rows Nleft..; blocked / blocked_r: mvpMapPoints[idx] (resp. [Nleft + idx]) with
        Observations() > 0 on entry; l2r / r2l: mvLeftToRightMatch / mvRightToLeftMatch; per MapPoint: flags
        (bit0 searched left, bit1 Observations() > 0, bit2 searched right), proj (n x 4: mTrackProjX,
        mTrackProjY, -, mTrackViewCos), mnTrackScaleLevel, proj_r (mTrackProjXR, mTrackProjYR, -,
        mTrackViewCosR), mnTrackScaleLevelR, descriptor.  Returns (nmatches, match, match_r)."""
        params.nnratio = self.nnratio
        k = np.ascontiguousarray(kps).view(KEYPOINT_DTYPE)
        kr = np.ascontiguousarray(kps_r).view(KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        dr = np.ascontiguousarray(desc_r, np.uint8).reshape(-1, 32)
        fl = np.ascontiguousarray(mp_flags, np.uint8)
        pr = np.ascontiguousarray(mp_proj, np.float32).reshape(-1, 4)
        lv = np.ascontiguousarray(mp_level, np.int32)
        prr = np.ascontiguousarray(mp_proj_r, np.float32).reshape(-1, 4)
        lvr = np.ascontiguousarray(mp_level_r, np.int32)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        opt = lambda a, t: None if a is None else np.ascontiguousarray(a, t)  # noqa: E731
        cb, cbr, a, b = opt(blocked, np.uint8), opt(blocked_r, np.uint8), opt(l2r, np.int32), opt(r2l, np.int32)
        pp = lambda a: None if a is None else _ptr(a)  # noqa: E731
        out = np.full(max(len(k), 1), -1, np.int32)
        outr = np.full(max(len(kr), 1), -1, np.int32)
        nm = _check(self._lib.plvi_search_local_stereo(ctypes.byref(params), _ptr(k), _ptr(d), len(k), pp(cb), pp(a),
                                                       _ptr(kr), _ptr(dr), len(kr), pp(cbr), pp(b), _ptr(fl), _ptr(pr),
                                                       _ptr(lv), _ptr(prr), _ptr(lvr), _ptr(md), len(fl), _ptr(out),
                                                       _ptr(outr)),
                    "plvi_search_local_stereo")
        return nm, out[:len(k)], outr[:len(kr)]

    def SearchByProjectionKF(self, params, cur_kps, cur_desc, kf_flags, x3dc, dist, level, kf_angle, mp_desc,
                             cur_blocked=None):
        """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:2180-2300),
        the relocalization guided search, with mbCheckOrientation = checkOri of this matcher.  params:
        RelocParams (camera, bounds, grid, th, orb_dist, scale factors); cur_kps: mvKeysUn; cur_blocked:
        mvpMapPoints[i2] != NULL on entry; per KF MapPoint (GetMapPointMatches() order): flags (bit0 = live and
        not in sAlreadyFound), x3dc (n x 3), dist (n x 3: dist3D, min / max distance invariance), level
        (PredictScale), kf_angle (pKF->mvKeysUn[i].angle), descriptor.  Returns (nmatches, match) with
        match[i2] = KF MapPoint index, -2 (nulled by the rotation filter) or -1 (untouched)."""
        params.check_orientation = int(self.check_orientation)
        ck = np.ascontiguousarray(cur_kps).view(KEYPOINT_DTYPE)
        cd = np.ascontiguousarray(cur_desc, np.uint8).reshape(-1, 32)
        n = len(ck)
        fl = np.ascontiguousarray(kf_flags, np.uint8)
        x3 = np.ascontiguousarray(x3dc, np.float32).reshape(-1, 3)
        ds = np.ascontiguousarray(dist, np.float32).reshape(-1, 3)
        lv = np.ascontiguousarray(level, np.int32)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        cb = None if cur_blocked is None else np.ascontiguousarray(cur_blocked, np.uint8)
        out = np.full(max(n, 1), -1, np.int32)
        nm = _check(self._lib.plvi_search_reloc(ctypes.byref(params), _ptr(ck), _ptr(cd), n,
                                                None if cb is None else _ptr(cb), _ptr(fl), _ptr(x3), _ptr(ds),
                                                _ptr(lv), _ptr(ka), _ptr(md), len(fl), _ptr(out)),
                    "plvi_search_reloc")
        return nm, out[:n]

    @staticmethod
    def DescriptorDistance(a, b, line_matcher_quirk=False):
        """Row-wise distances of two n x 32 descriptor tables on the GPU."""
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        n = a.shape[0]
        lib = load()
        da, db, do = DeviceBuffer(max(a.nbytes, 32)), DeviceBuffer(max(b.nbytes, 32)), DeviceBuffer(max(4 * n, 4))
        da.upload(a)
        db.upload(b)
        _check(lib.plvi_descriptor_distance_batch(ctypes.c_void_p(da.ptr), ctypes.c_void_p(db.ptr), n,
                                                  int(line_matcher_quirk), ctypes.c_void_p(do.ptr), None),
               "plvi_descriptor_distance_batch")
        lib.plvi_device_synchronize()
        return do.download(np.zeros(n, np.int32))


def frame_extract_batch(orb, lines, d_frames_ptr, n_frames, frame_stride, row_stride, lap=(0, 0), stream=None):
    """Frame::Frame's ORB + line extraction of a device batch as one schedule
    (plvi_frame_extract_batch); results via orb.outputs() / lines.outputs()."""
    _check(load().plvi_frame_extract_batch(orb._h, lines._h, ctypes.c_void_p(d_frames_ptr), n_frames, frame_stride,
                                           row_stride, lap[0], lap[1], ctypes.c_void_p(stream or 0)),
           "plvi_frame_extract_batch")


def frame_extract_match_batch(orb, lines, d_frames_ptr, n_frames, frame_stride, row_stride, knn_out, nnr,
                              line_scratch, line_matches, line_nmatch, lap=(0, 0), stream=None):
    """plvi_frame_extract_match_batch: the frame schedule plus the step's matching of frame t vs t-1 (ORB
    kNN-2 into knn_out = (idx0, d0, idx1, d1) device pointers, LineMatcher::match into line_matches /
    line_nmatch) issued inside the schedule's streams."""
    V = ctypes.c_void_p
    _check(load().plvi_frame_extract_match_batch(orb._h, lines._h, V(d_frames_ptr), n_frames, frame_stride, row_stride,
                                                 lap[0], lap[1], *[V(p) for p in knn_out], ctypes.c_float(nnr),
                                                 V(line_scratch), V(line_matches), V(line_nmatch), V(stream or 0)),
           "plvi_frame_extract_match_batch")


def frame_orb_event(lines):
    """plvi_frame_orb_event: the hipEvent_t the last frame_extract_batch on `lines` recorded when its ORB
    part completed (handle-owned)."""
    e = ctypes.c_void_p()
    _check(load().plvi_frame_orb_event(lines._h, ctypes.byref(e)), "plvi_frame_orb_event")
    return e.value


def event_create():
    e = ctypes.c_void_p()
    _check(load().plvi_event_create(ctypes.byref(e)), "plvi_event_create")
    return e.value


def event_record(event, stream=None):
    _check(load().plvi_event_record(ctypes.c_void_p(event), ctypes.c_void_p(stream or 0)), "plvi_event_record")


def stream_wait_event(stream, event):
    _check(load().plvi_stream_wait_event(ctypes.c_void_p(stream or 0), ctypes.c_void_p(event)),
           "plvi_stream_wait_event")


def event_destroy(event):
    _check(load().plvi_event_destroy(ctypes.c_void_p(event)), "plvi_event_destroy")


def stereo_frame_extract_batch(orb_left, orb_right, lines_left, lines_right, d_left_ptr, d_right_ptr, n_frames,
                               frame_stride, row_stride, lap=(0, 0), stream=None):
    """The stereo-line Frame's four extractions (plvi_stereo_frame_extract_batch)."""
    V = ctypes.c_void_p
    _check(load().plvi_stereo_frame_extract_batch(orb_left._h, orb_right._h, lines_left._h, lines_right._h,
                                                  V(d_left_ptr), V(d_right_ptr), n_frames, frame_stride, row_stride,
                                                  lap[0], lap[1], V(stream or 0)), "plvi_stereo_frame_extract_batch")


class StepGraph:
    """A batch step captured into a HIP graph (plvi_graph_*): ``fn(stream)``
    issues plvi_* calls on ``stream`` (a created stream); the graph replays
    them with one launch.  The captured pointers and parameters are fixed."""

    def __init__(self, fn, stream):
        self._lib = load()
        self._stream = stream
        _check(self._lib.plvi_graph_capture_begin(ctypes.c_void_p(stream)), "plvi_graph_capture_begin")
        try:
            fn(stream)
        finally:
            ex = ctypes.c_void_p()
            rc = self._lib.plvi_graph_capture_end(ctypes.c_void_p(stream), ctypes.byref(ex))
        _check(rc, "plvi_graph_capture_end")
        self._exec = ex

    def launch(self, stream=None):
        _check(self._lib.plvi_graph_launch(self._exec, ctypes.c_void_p(stream or self._stream)), "plvi_graph_launch")

    def __del__(self):
        if getattr(self, "_exec", None):
            self._lib.plvi_graph_destroy(self._exec)
            self._exec = None


class ORBVocabulary:
    """DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary.h) on the GPU.

    ``ORBVocabulary.loadFromTextFile(path)`` mirrors the reference loader
    (TemplatedVocabulary.h:1338-1424); ``ORBVocabulary.from_nodes(...)`` builds
    the same structure from a node table.  ``transform(desc, levelsup)``
    returns ``(BowVector, FeatureVector)`` as dicts {word: value} and
    {node: [feature indices]} in std::map (ascending key) order
    (TemplatedVocabulary.h:1126-1194).
    """

    def __init__(self, handle):
        self._lib = load()
        self._h = handle
        info = np.zeros(6, np.int32)
        _check(self._lib.plvi_vocab_info(self._h, _ptr(info)), "plvi_vocab_info")
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = (int(x) for x in info)

    @classmethod
    def loadFromTextFile(cls, path, emulate_tail=False, device=0):
        """TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424).  emulate_tail=True adds
        the node the reference's `while(!f.eof()) getline` loop reads from the empty tail after a final
        newline -- undefined in the reference (pid / nIsLeaf / the descriptor stay unassigned), modelled here
        as a zero-descriptor non-word child of the root; off by default."""
        h = ctypes.c_void_p()
        _check(load().plvi_vocab_load_text(str(path).encode(), int(emulate_tail), device, ctypes.byref(h)),
               "plvi_vocab_load_text")
        return cls(h)

    @classmethod
    def from_nodes(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device=0):
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        h = ctypes.c_void_p()
        _check(load().plvi_vocab_create(k, L, scoring, weighting, len(parent), _ptr(parent), _ptr(is_leaf),
                                        _ptr(desc), _ptr(weight), device, ctypes.byref(h)), "plvi_vocab_create")
        return cls(h)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.plvi_vocab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def empty(self):
        return self.n_words == 0

    def transform_arrays(self, desc, levelsup=4):
        """Raw CSR form: (bow_word, bow_value, fv_node, fv_off, fv_idx)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = d.shape[0]
        m = max(n, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fo, fi = np.zeros(m, np.uint32), np.zeros(m + 1, np.int32), np.zeros(m, np.uint32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        _check(self._lib.plvi_vocab_transform(self._h, _ptr(d), n, levelsup, _ptr(bw), _ptr(bv), ctypes.byref(nb),
                                              _ptr(fn), _ptr(fo), _ptr(fi), ctypes.byref(nf)), "plvi_vocab_transform")
        nb, nf = nb.value, nf.value
        return bw[:nb], bv[:nb], fn[:nf], fo[:nf + 1], fi[:fo[nf]]

    def transform(self, desc, levelsup=4):
        bw, bv, fn, fo, fi = self.transform_arrays(desc, levelsup)
        bow = {int(w): float(v) for w, v in zip(bw, bv)}
        fv = {int(fn[i]): [int(x) for x in fi[fo[i]:fo[i + 1]]] for i in range(len(fn))}
        return bow, fv

    def transform_features(self, desc, levelsup=4):
        """Per-descriptor (word ids, node ids at level L - levelsup)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = d.shape[0]
        w, ni = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint32)
        _check(self._lib.plvi_vocab_transform_features(self._h, _ptr(d), n, levelsup, _ptr(w), _ptr(ni)),
               "plvi_vocab_transform_features")
        return w[:n], ni[:n]


def assign_grid_batch(d_kps, d_count, cap, n_frames, grid, d_cell_off, d_cell_idx, stream=None):
    """Frame::AssignFeaturesToGrid (src/Frame.cc:644-675) of device keypoint tables -> CSR grids."""
    _check(load().plvi_assign_grid_batch(ctypes.c_void_p(d_kps), ctypes.c_void_p(d_count), cap, n_frames,
                                         ctypes.byref(grid), ctypes.c_void_p(d_cell_off),
                                         ctypes.c_void_p(d_cell_idx), ctypes.c_void_p(stream or 0)),
           "plvi_assign_grid_batch")


# ------------------------------------------------------- initialization
def search_for_initialization_batch(n_pairs, params, d_kps1, d_desc1, d_n1, cap1, d_prev, d_kps2, d_desc2, d_n2, cap2,
                                    d_cell_off, d_cell_idx, d_m12, d_nm, stream=None):
    """ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:705-814) over device pair tables."""
    V = ctypes.c_void_p
    _check(load().plvi_search_for_initialization_batch(n_pairs, ctypes.byref(params), V(d_kps1), V(d_desc1), V(d_n1),
                                                       cap1, V(d_prev), V(d_kps2), V(d_desc2), V(d_n2), cap2,
                                                       V(d_cell_off), V(d_cell_idx), V(d_m12), V(d_nm),
                                                       V(stream or 0)),
           "plvi_search_for_initialization_batch")


def search_for_initialization(kps1, desc1, prev_xy, kps2, desc2, width=640, height=480, window=100, nnratio=0.9,
                              check_orientation=True, grid=None):
    """One (F1, F2) pair from host arrays (keypoints in KEYPOINT_DTYPE = mvKeysUn,
    descriptors n x 32, prev_xy = vbPrevMatched n1 x 2): returns (nmatches,
    vnMatches12, updated vbPrevMatched).  grid = (min_x, min_y, inv_w, inv_h)
    (default: the Frame grid of an undistorted width x height image)."""
    n1, n2 = len(kps1), len(kps2)
    if grid is None:
        g = grid_geometry(width, height)
        grid = (g[0], g[2], g[4], g[5])
    p = InitParams(float(grid[0]), float(grid[1]), float(grid[2]), float(grid[3]), int(window), float(nnratio),
                   int(bool(check_orientation)))
    c1, c2 = max(n1, 1), max(n2, 1)
    k1 = np.zeros(c1, KEYPOINT_DTYPE)
    k1[:n1] = kps1
    k2 = np.zeros(c2, KEYPOINT_DTYPE)
    k2[:n2] = kps2
    d1 = np.zeros((c1, 32), np.uint8)
    d1[:n1] = desc1
    d2 = np.zeros((c2, 32), np.uint8)
    d2[:n2] = desc2
    pv = np.zeros((c1, 2), np.float32)
    pv[:n1] = prev_xy
    bufs = [DeviceBuffer(a.nbytes) for a in (k1, d1, pv, k2, d2)]
    for b, a in zip(bufs, (k1, d1, pv, k2, d2)):
        b.upload(a)
    cnt = DeviceBuffer(16)
    cnt.upload(np.array([n1, n2, 0, 0], np.int32))
    co = DeviceBuffer(4 * 3073)
    ci = DeviceBuffer(4 * c2)
    m = DeviceBuffer(4 * c1)
    assign_grid_batch(bufs[3].ptr, cnt.ptr + 4, c2, 1, GridParams(*[float(v) for v in grid]), co.ptr, ci.ptr)
    search_for_initialization_batch(1, p, bufs[0].ptr, bufs[1].ptr, cnt.ptr, c1, bufs[2].ptr, bufs[3].ptr, bufs[4].ptr,
                                    cnt.ptr + 4, c2, co.ptr, ci.ptr, m.ptr, cnt.ptr + 8)
    load().plvi_device_synchronize()
    out = cnt.download(np.zeros(4, np.int32))
    return int(out[2]), m.download(np.zeros(c1, np.int32))[:n1], bufs[2].download(np.zeros((c1, 2), np.float32))[:n1]


def line_search_init_batch(d_desc1, d_n1, cap1, d_desc2, d_n2, cap2, n_pairs, d_scratch, d_pairs, d_npairs, d_mad=0,
                           stream=None):
    """LineMatcher::SerachForInitialize + Frame::lineDescriptorMAD over device pair tables."""
    V = ctypes.c_void_p
    _check(load().plvi_line_search_init_batch(V(d_desc1), V(d_n1), cap1, V(d_desc2), V(d_n2), cap2, n_pairs,
                                              V(d_scratch), V(d_pairs), V(d_npairs), V(d_mad), V(stream or 0)),
           "plvi_line_search_init_batch")


def line_search_init(desc1, desc2):
    """One pair from host arrays: returns (LineMatches as an n x 2 int array
    (query, train), (nn_mad, nn12_mad))."""
    n1, n2 = len(desc1), len(desc2)
    c1, c2 = max(n1, 1), max(n2, 1)
    d1 = np.zeros((c1, 32), np.uint8)
    d1[:n1] = desc1
    d2 = np.zeros((c2, 32), np.uint8)
    d2[:n2] = desc2
    b1, b2 = DeviceBuffer(d1.nbytes), DeviceBuffer(d2.nbytes)
    b1.upload(d1)
    b2.upload(d2)
    cnt = DeviceBuffer(16)
    cnt.upload(np.array([n1, n2, 0, 0], np.int32))
    scr = DeviceBuffer(16 * c1)
    pr = DeviceBuffer(8 * c1)
    mad = DeviceBuffer(16)
    line_search_init_batch(b1.ptr, cnt.ptr, c1, b2.ptr, cnt.ptr + 4, c2, 1, scr.ptr, pr.ptr, cnt.ptr + 8, mad.ptr)
    load().plvi_device_synchronize()
    n = int(cnt.download(np.zeros(4, np.int32))[2])
    return pr.download(np.zeros((c1, 2), np.int32))[:n], tuple(mad.download(np.zeros(2, np.float64)))


# ----------------------------------------------------------------- stereo
def pack_pyramid(levels):
    """mvImagePyramid (list of 2-D uint8 arrays) -> (concatenated bytes, offsets, widths, heights)."""
    off = np.zeros(len(levels), np.int64)
    o = 0
    for i, lv in enumerate(levels):
        off[i] = o
        o += lv.size
    buf = np.concatenate([np.ascontiguousarray(lv, np.uint8).ravel() for lv in levels])
    w = np.array([lv.shape[1] for lv in levels], np.int32)
    h = np.array([lv.shape[0] for lv in levels], np.int32)
    return buf, off, w, h


def ComputeStereoMatches(kpsL, descL, kpsR, descR, pyrL, pyrR, scale_factors, inv_scale_factors, mb, mbf):
    """Frame::ComputeStereoMatches (src/Frame.cc:1228-1406) for one rectified pair.  kps*: mvKeys /
    mvKeysRight (KEYPOINT_DTYPE), pyr*: mvImagePyramid of the left / right extractor.  Returns
    (nstereo, mvuRight, mvDepth)."""
    lib = load()
    kl = np.ascontiguousarray(kpsL).view(KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kpsR).view(KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(descL, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(descR, np.uint8).reshape(-1, 32)
    bl, off, w, h = pack_pyramid(pyrL)
    br, off2, w2, h2 = pack_pyramid(pyrR)
    if not (np.array_equal(off, off2) and np.array_equal(w, w2) and np.array_equal(h, h2)):
        raise ValueError("left and right pyramids differ in geometry")
    sc = np.ascontiguousarray(scale_factors, np.float32)
    inv = np.ascontiguousarray(inv_scale_factors, np.float32)
    n = len(kl)
    ur = np.full(max(n, 1), -1, np.float32)
    dp = np.full(max(n, 1), -1, np.float32)
    k = _check(lib.plvi_stereo_match(_ptr(kl), _ptr(dl), n, _ptr(kr), _ptr(dr), len(kr), len(pyrL), _ptr(sc),
                                     _ptr(inv), _ptr(bl), _ptr(br), _ptr(off), _ptr(w), _ptr(h), float(mb),
                                     float(mbf), _ptr(ur), _ptr(dp)), "plvi_stereo_match")
    return k, ur[:n], dp[:n]


def stereo_match_batch(left, right, n_frames, mb, mbf, d_uright, d_depth, d_nstereo, d_err, stream=None):
    """plvi_stereo_match_batch on two ORBextractor handles (device outputs, asynchronous)."""
    _check(load().plvi_stereo_match_batch(left._h, right._h, n_frames, float(mb), float(mbf),
                                          ctypes.c_void_p(d_uright), ctypes.c_void_p(d_depth),
                                          ctypes.c_void_p(d_nstereo), ctypes.c_void_p(d_err),
                                          ctypes.c_void_p(stream or 0)), "plvi_stereo_match_batch")


def ComputeStereoMatches_Lines(klL, descL, klR, descR, klUn, width, height, mbf, range_hint=1):
    """Frame::ComputeStereoMatches_Lines (src/Frame.cc:1408-1492) for one pair: mvKeys_Line, mvKeysRight_Line,
    mvKeysUn_Line (KEYLINE_DTYPE), LBD descriptors.  Returns (nstereo, matches_12, mvDisparity_l (n x 2),
    mvDepth_l (n x 2), mvle_l (n x 3))."""
    lib = load()
    a = np.ascontiguousarray(klL).view(KEYLINE_DTYPE)
    b = np.ascontiguousarray(klR).view(KEYLINE_DTYPE)
    u = a if klUn is None else np.ascontiguousarray(klUn).view(KEYLINE_DTYPE)
    dl = np.ascontiguousarray(descL, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(descR, np.uint8).reshape(-1, 32)
    n = len(a)
    m = np.full(max(n, 1), -1, np.int32)
    disp = np.full((max(n, 1), 2), -1, np.float32)
    dep = np.full((max(n, 1), 2), -1, np.float32)
    le = np.zeros((max(n, 1), 3), np.float64)
    k = _check(lib.plvi_stereo_lines(_ptr(a), _ptr(dl), n, _ptr(b), _ptr(dr), len(b), _ptr(u), int(width),
                                     int(height), float(mbf), int(range_hint), _ptr(m), _ptr(disp), _ptr(dep),
                                     _ptr(le)), "plvi_stereo_lines")
    return k, m[:n], disp[:n], dep[:n], le[:n]


def stereo_lines_scratch_bytes(n_frames, capL, capR, idx_cap):
    return load().plvi_stereo_lines_scratch_bytes(n_frames, capL, capR, idx_cap)


def stereo_lines_batch(n_frames, d_klL, d_descL, d_nL, capL, d_klR, d_descR, d_nR, capR, d_klUn, width, height,
                       mbf, range_hint, idx_cap, d_scratch, scratch_bytes, d_m12, d_disp, d_depth, d_le, d_nstereo,
                       d_err, stream=None):
    """plvi_stereo_lines_batch on device keyline tables (asynchronous)."""
    V = ctypes.c_void_p
    _check(load().plvi_stereo_lines_batch(n_frames, V(d_klL), V(d_descL), V(d_nL), capL, V(d_klR), V(d_descR),
                                          V(d_nR), capR, V(d_klUn or 0), width, height, float(mbf), range_hint,
                                          idx_cap, V(d_scratch), scratch_bytes, V(d_m12), V(d_disp), V(d_depth),
                                          V(d_le), V(d_nstereo), V(d_err), V(stream or 0)), "plvi_stereo_lines_batch")
