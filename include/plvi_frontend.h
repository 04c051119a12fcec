/* plvi_frontend.h — C-ABI of the MI355X-native PL-VI-ORBSLAM3 feature front end.
 *
 * Plain pointers and sizes only.  Each entry point replaces one reference
 * interface (cited per function); INTEGRATION.md gives the C++ shim bodies
 * a maintainer drops into the reference classes (ORBextractor,
 * Lineextractor, ORBmatcher, LineMatcher, ORBVocabulary), and
 * pl-vi-orbslam3_amd/plvi/ is the Python (ctypes) mirror.
 *
 * Status codes: 0 = ok, negative = error (PLVI_E_*).  ORBextractor's
 * "empty image -> -1" convention (src/ORBextractor.cc:1072-1073) is kept by
 * plvi_orb_extract returning PLVI_E_EMPTY (-1).
 *
 * Threading: handles are independent and may be used from
 * different host threads concurrently (each owns its device scratch and HIP
 * stream); one handle is not re-entrant, exactly like the reference
 * extractor whose operator() mutates mvImagePyramid.
 */
#ifndef PLVI_FRONTEND_H
#define PLVI_FRONTEND_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  PLVI_OK = 0,
  PLVI_E_EMPTY = -1,    /* empty image (ORBextractor.cc:1072) */
  PLVI_E_BADARG = -2,   /* bad size / parameter / type */
  PLVI_E_CAPACITY = -3, /* caller's output capacity too small (count still written) */
  PLVI_E_HIP = -4,      /* HIP runtime failure */
  PLVI_E_OVERFLOW = -5, /* internal fixed-capacity table overflowed on device */
  PLVI_E_SIZE = -6,     /* descriptor row counts differ (LineMatcher.cpp:50-51) */
  PLVI_E_CAPTURE = -7,  /* stream capture of the multi-stream frame schedule on a HIP runtime < 7.2 */
};

/* OpenCV-semantics switches for the items no reference test can pin
 * (confidence "M"); 0 = the default guesses.  Set in
 * plvi_orb_params.compat / plvi_line_params.compat at create time; the CPU
 * oracle takes the same flags.
 *  GAUSS_ROUNDED   A.4: GaussianBlur CV_8U taps by plain rounding
 *                  ([18,34,49,55,49,34,18] for 7x7 sigma 2, ORBextractor.cc:1115;
 *                  [14,63,103,63,14] for 5x5 sigma 1, binary_descriptor_custom.cpp:359)
 *                  instead of the error-diffused [18,34,48,56,..] / [14,62,104,..]
 *  RESIZE_V_GENERIC A.1: cv::resize INTER_LINEAR 8U vertical pass by the generic
 *                  (b0*H0 + b1*H1 + (1<<21)) >> 22 instead of the 8U
 *                  specialisation ((b0*(H0>>4))>>16 + (b1*(H1>>4))>>16 + 2) >> 2
 *                  (ORBextractor.cc:1165)
 *  EXP_CV_TABLE    A.6: the f64 7-tap LSD Gaussian (lsd.cpp:455) built with
 *                  OpenCV's table + polynomial exp (EXPTAB_SCALE 6) instead of
 *                  glibc exp (which equals the correctly rounded exp there)
 *  GEMM_FMA        the pose product Rcw*P + tcw of the frustum tests (cv::gemm,
 *                  3x3 * 3x1 + 3x1 float) as OpenCV's AVX2-dispatched build
 *                  contracts it, fma(a2,b2, fma(a0,b0, a1*b1)), instead of the
 *                  baseline (a0*b0 + a1*b1) + a2*b2 (plvi_frustum_params.compat) */
enum {
  PLVI_COMPAT_GAUSS_ROUNDED = 1,
  PLVI_COMPAT_RESIZE_V_GENERIC = 2,
  PLVI_COMPAT_EXP_CV_TABLE = 4,
  PLVI_COMPAT_GEMM_FMA = 8,
};

/* Per-frame device error flags of a batch (plvi_orb_errors / plvi_lines_errors). */
enum {
  PLVI_FERR_OCTREE = 1,   /* ORB: an octree level exceeded its node table (level dropped) */
  PLVI_FERR_LSD_TILE = 2, /* lines: reserved (the streaming LSD prep has no tile to overflow) */
  PLVI_FERR_LSD_RAW = 4,  /* lines: more LSD regions than the raw line table holds */
  PLVI_FERR_KEYLINES = 8, /* lines: keyline table overflow (frame emitted with 0 lines) */
};

/* cv::KeyPoint layout (28 bytes): pt.x, pt.y, size, angle, response, octave, class_id. */
typedef struct plvi_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} plvi_keypoint;

/* cv::line_descriptor::KeyLine layout (descriptor_custom.hpp:107-146). */
typedef struct plvi_keyline {
  float angle;
  int32_t class_id;
  int32_t octave;
  float pt_x, pt_y;
  float response;
  float size;
  float startPointX, startPointY, endPointX, endPointY;
  float sPointInOctaveX, sPointInOctaveY, ePointInOctaveX, ePointInOctaveY;
  float lineLength;
  int32_t numOfPixels;
} plvi_keyline;

/* ------------------------------------------------------------------ ORB
 * Replaces ORB_SLAM3::ORBextractor (include/ORBextractor.h:44-110,
 * src/ORBextractor.cc:408-1177). */
typedef struct plvi_orb_extractor plvi_orb_extractor;

typedef struct plvi_orb_params {
  int nfeatures;      /* ORBextractor(int nfeatures, ...) */
  float scale_factor; /* float scaleFactor (stored as double, .h:97) */
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
  unsigned compat;    /* PLVI_COMPAT_* (0 = defaults) */
} plvi_orb_params;

/* Create an extractor for frames of width x height, batches of up to
 * max_batch frames, on HIP device `device`.  Replaces the constructor
 * (ORBextractor.cc:408-468). */
int plvi_orb_create(const plvi_orb_params* p, int width, int height, int max_batch, int device,
                    plvi_orb_extractor** out);
int plvi_orb_destroy(plvi_orb_extractor* h);

/* One frame from host memory, synchronous: ORBextractor::operator()
 * (ORBextractor.cc:1068-1150).  Keypoints are written in the reference's
 * slot order (mono slots ascending from 0, vLappingArea slots from the back);
 * descriptors are n x 32 bytes in the same row order.  *n = number of
 * keypoints, *mono_index = return value of operator() (monoIndex).
 * Returns PLVI_E_EMPTY for an empty image.  Like operator() it accepts any
 * frame size: a size other than the handle's re-plans the handle (pyramid,
 * cells, buffers) for the new size, which the batch entry points then use. */
int plvi_orb_extract(plvi_orb_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                     int lap0, int lap1, plvi_keypoint* kps, uint8_t* desc, int cap, int* n, int* mono_index);

/* Batched, device-resident variant: n_frames frames at d_frames (device
 * pointer, frame f row r at d_frames + f*frame_stride + r*row_stride), all
 * of the handle's width x height.  Asynchronous on `stream` (hipStream_t,
 * NULL = the handle's own stream).  Results stay on the device: see
 * plvi_orb_outputs. */
int plvi_orb_extract_batch(plvi_orb_extractor* h, const uint8_t* d_frames, int n_frames, size_t frame_stride,
                           size_t row_stride, int lap0, int lap1, void* stream);

/* Device error flags of the batches run since the last call (PLVI_FERR_*),
 * read and cleared: frame_flags[f] for frame slot f (max_batch ints, may be
 * NULL), *any = OR over all slots (may be NULL).  Synchronises `stream`
 * (NULL = the handle's stream), on which the flags are read and reset.  A
 * frame with a flag set has truncated tables; the single-frame entry
 * points report the same condition as PLVI_E_OVERFLOW. */
int plvi_orb_errors(plvi_orb_extractor* h, int* frame_flags, int* any, void* stream);

/* Device pointers to the last batch's outputs: keypoints [max_batch][cap],
 * descriptors [max_batch][cap][32], counts [max_batch], mono [max_batch].
 * *cap = per-frame keypoint capacity (sum of per-level octree capacities). */
int plvi_orb_outputs(plvi_orb_extractor* h, plvi_keypoint** d_kps, uint8_t** d_desc, int** d_count, int** d_mono,
                     int* cap);

/* mvImagePyramid[level] of frame `frame` of the last call (lazy D2H copy).
 * dst must hold w*h bytes; pass dst=NULL to query the size.  Level 0 is read
 * from the last call's input frames when they were packed (see
 * plvi_orb_pyramid_device), so call this before they are overwritten. */
int plvi_orb_pyramid_level(plvi_orb_extractor* h, int frame, int level, uint8_t* dst, int* w, int* hgt);

/* Device view of mvImagePyramid (include/ORBextractor.h:84, read by
 * Frame::ComputeStereoMatches, src/Frame.cc:1235,1325,1344): level `level`
 * of frame f is the w x hgt u8 image (row stride w) at
 * *d_frame0 + f * *frame_stride, valid after the last extraction on the
 * handle's stream.  Level 0 is the input image itself (ORBextractor.cc:1165
 * copies it unchanged): when the last batch's rows were packed (row_stride ==
 * width) it is returned as a view of the caller's frames (the batch pointer and
 * its frame_stride; plvi_orb_extract's own staging copy for single frames),
 * valid while that buffer is unchanged; otherwise the handle holds a copy.
 * level = -1 only reports *nlevels.  Any out pointer may be NULL. */
int plvi_orb_pyramid_device(plvi_orb_extractor* h, int level, const uint8_t** d_frame0, size_t* frame_stride, int* w,
                            int* hgt, int* nlevels);

/* GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (include/ORBextractor.h:62-82): nlevels floats each. */
int plvi_orb_scale_tables(plvi_orb_extractor* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2);

/* Per-level feature quota (mnFeaturesPerLevel, ORBextractor.cc:433-444). */
int plvi_orb_level_quota(plvi_orb_extractor* h, int* quota);

/* Stage timing (HIP events on the launch stream) for bench.py's roofline:
 * enable=1 resets and starts recording, 0 stops.  profile_read synchronises
 * and returns per-stage milliseconds summed over the recorded runs (up to
 * 512): [0] level build (resize+blur+FAST score), [1] cell NMS, [2] SAT,
 * [3] octree, [4] node best, [5] orientation+rBRIEF, [6] output assembly. */
int plvi_orb_profile(plvi_orb_extractor* h, int enable);
int plvi_orb_profile_read(plvi_orb_extractor* h, float* stage_ms, int* runs);

/* Per-launch timing of the pyramid blur + FAST kernel (bench.py's roofline
 * kernel) and of the pyramid kernel: enable=1 resets and records an event pair around every launch on
 * its launch stream (up to 4096 launches); read synchronises and returns the
 * summed milliseconds and the launch count. */
int plvi_orb_kernel_timing(plvi_orb_extractor* h, int enable);
int plvi_orb_kernel_timing_read(plvi_orb_extractor* h, float* total_ms, int* launches);
/* The same for kind 0 = blur + FAST, 1 = orb_pyramid_kernel (roofline_pyramid). */
int plvi_orb_kernel_timing_read_kind(plvi_orb_extractor* h, int kind, float* total_ms, int* launches);
/* Diagnostic: cap every level's octree node capacity at `cap` (<= 0 restores
 * the planned capacities).  A level whose DistributeOctTree needs more nodes
 * flags its frame (plvi_orb_errors bit 1) and yields no keypoints; the test
 * hook for that path. */
int plvi_orb_debug_node_cap(plvi_orb_extractor* h, int cap);

/* ------------------------------------------------------------------ Lines
 * Replaces ORB_SLAM3::Lineextractor (include/LineExtractor.h:49-93,
 * src/LineExtractor.cc:39-117): LSDDetectorC pyramid + LSD
 * (src/LSD/lsd.cpp) + KeyLine assembly + top-k + LBD
 * (Thirdparty/line_descriptor/src/binary_descriptor_custom.cpp). */
typedef struct plvi_line_extractor plvi_line_extractor;

typedef struct plvi_line_params {
  int nfeatures;   /* lsd_nfeatures (0 = keep all) */
  int refine;      /* lsd_refine: only 0 (LSD_REFINE_NONE, the config) is supported */
  float lsd_scale; /* lsd_scale (LSDOptions::scale, float) */
  int nlevels;     /* pyramid octaves (<= 2) */
  float scale;     /* pyramid scale factor (2.0) */
  int extractor;   /* 0 = LSD (EDLines, extractor==1, is out of scope) */
  unsigned compat; /* PLVI_COMPAT_* (0 = defaults) */
} plvi_line_params;

int plvi_lines_create(const plvi_line_params* p, int width, int height, int max_batch, int device,
                      plvi_line_extractor** out);
int plvi_lines_destroy(plvi_line_extractor* h);

/* One frame from host memory, synchronous: Lineextractor::operator()
 * (LineExtractor.cc:45-117).  keylines (KeyLine layout) in the reference's
 * order (post top-k sort when truncated), LBD descriptors n x 32, and the
 * normalised line equations n x 3 doubles (keylineFunction).  The reference
 * APPENDS to keylineFunction; callers append line_fns themselves. Any frame
 * size is accepted (re-plans the handle, as for plvi_orb_extract). */
int plvi_lines_extract(plvi_line_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                       plvi_keyline* keylines, uint8_t* desc, double* line_fns, int cap, int* n);

/* Batched device-resident variant (same frame addressing as ORB). */
int plvi_lines_extract_batch(plvi_line_extractor* h, const uint8_t* d_frames, int n_frames, size_t frame_stride,
                             size_t row_stride, void* stream);
int plvi_lines_outputs(plvi_line_extractor* h, plvi_keyline** d_kl, uint8_t** d_desc, double** d_fn, int** d_count,
                       int* cap);
/* Per-frame device error flags (PLVI_FERR_*), read and cleared; as plvi_orb_errors. */
int plvi_lines_errors(plvi_line_extractor* h, int* frame_flags, int* any, void* stream);

/* mvImagePyramid_l[level] (gaussianPyrs, level >= 1; level 0 is the input). */
int plvi_lines_pyramid_level(plvi_line_extractor* h, int frame, int level, uint8_t* dst, int* w, int* hgt);

/* mvScaleFactor_l / mvInvScaleFactor_l / mvLevelSigma2_l / mvInvLevelSigma2_l (LineExtractor.cc:86-100). */
int plvi_lines_scale_tables(plvi_line_extractor* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2);

/* Stage timing: [0] octave pyramid, [1] LSD prep (blur f64, resize, gradient),
 * [2] region growing + rect, [3] keyline assembly + top-k, [4] LBD. */
int plvi_lines_profile(plvi_line_extractor* h, int enable);
/* Diagnostic cycle accounting inside the region-growing kernel (s_memtime):
 * per (frame, octave) 24 uint64 = [total, block setup, rounds, rect, seeds,
 * blocks, rounds, rect points, commits, 4 round phases, seed scan, seed
 * starts, init, HW_ID, XCC_ID, start time, -]; NULL disables. */
int plvi_lines_debug_stats(plvi_line_extractor* h, unsigned long long* d_stats);
/* Diagnostic counters of the multi-wave (small-batch) region-growing kernel:
 * per (frame, octave) 16 int32 = [regions dispatched speculatively, dropped,
 * regrown after a failed validation, grown exactly by the walk (never
 * dispatched), trivial seeds, speculative regions committed, walk cycles,
 * walker growth cycles, walk entries, walks blocked on a growing head seed,
 * kernel cycles, speculative growth cycles, idle polls, 0, 0, 0]; NULL
 * disables.  Batches up to PLVI_GROW_MW frames (default 256) take that kernel. */
int plvi_lines_debug_mw_stats(plvi_line_extractor* h, int* d_stats);
/* Diagnostic: LSD planes of the last batch for one (frame, octave), copied to
 * host: angle in degrees (float, NOTDEF = -1024), modgrad (f64), cos/sin
 * pairs (float2, defined pixels only); any pointer may be NULL. */
int plvi_lines_debug_planes(plvi_line_extractor* h, int frame, int octave, float* deg, double* modgrad, float* cs,
                            int* sw, int* sh);
/* Diagnostic: LBD Sobel plane of the last batch for one (frame, octave),
 * interleaved int16 (dx, dy) per pixel, copied to host; dxdy may be NULL. */
int plvi_lines_debug_sobel(plvi_line_extractor* h, int frame, int octave, short* dxdy, int* w, int* hgt);
int plvi_lines_profile_read(plvi_line_extractor* h, float* stage_ms, int* runs);
/* Per-launch timing of lsd_prep_kernel (bench.py's LSD-pass roofline), one
 * launch per octave: as plvi_orb_kernel_timing / _read. */
int plvi_lines_kernel_timing(plvi_line_extractor* h, int enable);
int plvi_lines_kernel_timing_read(plvi_line_extractor* h, float* total_ms, int* launches);
/* The same timing per kernel kind: 0 = lsd_prep_kernel, 1 = lbd_sobel0_kernel
 * (octave-0 5x5 blur + Sobel), 2 = lbd_sobel1_kernel (pyrDown + Sobel). */
int plvi_lines_kernel_timing_read_kind(plvi_line_extractor* h, int kind, float* total_ms, int* launches);

/* ------------------------------------------------------------------ Hamming
 * ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:2350-2366) over a batch. */

/* cv::BFMatcher(NORM_HAMMING).knnMatch(q, t, k=2) semantics (scan train rows
 * ascending, strict-< insertion): for each query i, idx0/d0 = best train row
 * and distance, idx1/d1 = second.  Missing entries are -1 / INT32_MAX.
 * Batched over n_pairs independent (query,train) pairs; all pointers device.
 * q: [n_pairs][nq_cap][32], t: [n_pairs][nt_cap][32]; nq/nt: per-pair counts
 * (device int arrays).  Outputs [n_pairs][nq_cap]. */
int plvi_hamming_knn2_batch(const uint8_t* d_q, const int* d_nq, int nq_cap, const uint8_t* d_t, const int* d_nt,
                            int nt_cap, int n_pairs, int* d_idx0, int* d_d0, int* d_idx1, int* d_d1, void* stream);

/* Host convenience wrapper (one pair, synchronous). */
int plvi_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* idx0, int* d0, int* idx1, int* d1);

/* LineMatcher::matchNNR (src/LineMatcher.cpp:41-61): matches_12[i] = train
 * index or -1; returns the number of matches (>=0) or an error code.
 * Requires nt >= 2 (the reference indexes matches_[idx][1]). */
int plvi_line_match_nnr(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr, int* matches_12);

/* LineMatcher::match(desc1, desc2, nnr, matches_12) (LineMatcher.cpp:92-111):
 * matchNNR both ways + mutual check. */
int plvi_line_match(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr, int* matches_12);

/* In/out variants with the reference's std::vector semantics: matches_12
 * holds the caller's n_prev existing entries on entry, and
 * matches_12.resize(n1, -1) (LineMatcher.cpp:44) keeps the first
 * min(n_prev, n1) of them (only accepted matches overwrite an entry) and
 * sets the rest to -1.  In plvi_line_match_inout a kept entry i2 >= 0 then
 * goes through the mutual check like a fresh one (LineMatcher.cpp:101-106);
 * a kept i2 >= n2 is out of range there (undefined in the reference) and
 * returns PLVI_E_BADARG. */
int plvi_line_match_nnr_inout(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr, int* matches_12,
                              int n_prev);
int plvi_line_match_inout(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr, int* matches_12,
                          int n_prev);

/* Batched LineMatcher::match on device descriptor tables: pair p matches
 * desc1[p] (n1[p] rows, stride cap1) against desc2[p] (n2[p] rows, stride
 * cap2).  d_scratch must hold 4*n_pairs*(cap1+cap2) ints.  Outputs
 * matches_12 [n_pairs][cap1] and per-pair match counts.  Pairs with fewer
 * than 2 rows on the train side produce no matches. */
int plvi_line_match_batch(const uint8_t* d_desc1, const int* d_n1, int cap1, const uint8_t* d_desc2, const int* d_n2,
                          int cap2, int n_pairs, float nnr, int* d_scratch, int* d_matches_12, int* d_nmatch,
                          void* stream);

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:2350-2366) or, with
 * line_matcher_quirk != 0, LineMatcher::DescriptorDistance
 * (src/LineMatcher.cpp:487-499: per-word count >> 25) of n row pairs
 * (d_a[i], d_b[i]), 32 bytes each; device pointers, asynchronous. */
int plvi_descriptor_distance_batch(const uint8_t* d_a, const uint8_t* d_b, int n, int line_matcher_quirk, int* d_out,
                                   void* stream);

/* ------------------------------------------------------------- SearchByBoW
 * ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&)
 * (src/ORBmatcher.cc:269-471) with ComputeThreeMaxima (:2304-2345),
 * monocular branch (F.Nleft == -1, no second camera).  FeatureVectors are
 * CSR arrays sorted by node id: node[i], off[i]..off[i+1] into idx[] (the
 * keypoint indices of node i in FeatureVector order).  kf_live[k] = the KF
 * keypoint has a MapPoint that is not bad (evaluated by the caller).
 * Angles: pKF->mvKeysUn[k].angle and F.mvKeys[i].angle.  Output
 * match_kf[i] = KF keypoint index whose MapPoint goes to
 * vpMapPointMatches[i], or -1.  Returns nmatches (>= 0) or an error. */
int plvi_search_by_bow(float nnratio, int check_orientation, const uint8_t* kf_desc, const float* kf_angle,
                       const uint8_t* kf_live, int kf_n, const int* kf_node, const int* kf_off, int kf_nnodes,
                       const int* kf_idx, const uint8_t* f_desc, const float* f_angle, int f_n, const int* f_node,
                       const int* f_off, int f_nnodes, const int* f_idx, int* match_kf);

/* Batched device variant: pair p uses rows p*kf_cap / p*f_cap of the
 * keypoint arrays, p*node_cap (node ids) and p*(node_cap+1) (offsets) of
 * the CSR arrays, counts kf_nnodes[p], f_nnodes[p], f_n[p].  Outputs
 * match_kf [n_pairs][f_cap], nmatches [n_pairs].  Needs
 * 4*f_cap + 8*node_cap <= 65536 bytes of LDS. */
int plvi_search_by_bow_batch(int n_pairs, float nnratio, int check_orientation, int kf_cap, int f_cap, int node_cap,
                             const uint8_t* d_kf_desc, const float* d_kf_angle, const uint8_t* d_kf_live,
                             const int* d_kf_node, const int* d_kf_off, const int* d_kf_nnodes, const int* d_kf_idx,
                             const uint8_t* d_f_desc, const float* d_f_angle, const int* d_f_n, const int* d_f_node,
                             const int* d_f_off, const int* d_f_nnodes, const int* d_f_idx, int* d_match_kf,
                             int* d_nmatches, void* stream);

/* The same with the two-camera branch of the reference (ORBmatcher.cc:321-420,
 * F.Nleft != -1: KannalaBrandt8 stereo rigs): keypoints [0, Nleft) are the
 * left camera's, [Nleft, N) the right one's (mvKeysRight); every KF keypoint
 * keeps a best / second pair per camera, and when the left best passes
 * TH_LOW the right best is also taken if it passes TH_LOW (its ratio test is
 * `|| true` in the reference).  Angles are per keypoint index as the
 * reference reads them (F: mvKeys for left indices, mvKeysRight[i - Nleft]
 * for right ones; KF: mvKeysUn without a second camera, else mvKeys /
 * mvKeysRight).  f_nleft = F.Nleft (-1 = one camera: plvi_search_by_bow);
 * d_f_nleft [n_pairs] (NULL = all -1). */
int plvi_search_by_bow_stereo(float nnratio, int check_orientation, const uint8_t* kf_desc, const float* kf_angle,
                              const uint8_t* kf_live, int kf_n, const int* kf_node, const int* kf_off, int kf_nnodes,
                              const int* kf_idx, const uint8_t* f_desc, const float* f_angle, int f_n,
                              const int* f_node, const int* f_off, int f_nnodes, const int* f_idx, int f_nleft,
                              int* match_kf);
int plvi_search_by_bow_stereo_batch(int n_pairs, float nnratio, int check_orientation, int kf_cap, int f_cap,
                                    int node_cap, const uint8_t* d_kf_desc, const float* d_kf_angle,
                                    const uint8_t* d_kf_live, const int* d_kf_node, const int* d_kf_off,
                                    const int* d_kf_nnodes, const int* d_kf_idx, const uint8_t* d_f_desc,
                                    const float* d_f_angle, const int* d_f_n, const int* d_f_node, const int* d_f_off,
                                    const int* d_f_nnodes, const int* d_f_idx, const int* d_f_nleft, int* d_match_kf,
                                    int* d_nmatches, void* stream);

/* ------------------------------------------------------------- matchGrid
 * LineMatcher::matchGrid(lines1, desc1, grid, desc2, directions2, w,
 * matches_12) (src/LineMatcher.cpp:191-272) with GridStructure::get
 * (src/gridStructure.cpp:64-75).  lines1: n1 x 4 ints (sp.x, sp.y, ep.x,
 * ep.y) = the line_2d grid coordinates (pair<int,int>, Frame.cc:1424-1427);
 * grid: CSR over grid_cols x grid_rows cells, cell (x, y) = x*grid_rows + y,
 * cell_off[ncell+1], cell_idx[] in std::list order; directions2: n2 x 2
 * doubles; window = GridWindow{width(w0, w1), height(h0, h1)}.
 * libstdcxx_range_hint selects the std::unordered_set range-insert rehash
 * rule that orders the candidates (1: GCC <= 10, the reference's Ubuntu
 * 20.04 toolchain; 0: GCC >= 11).  matches_12 is fully written (-1 = no
 * match).  Returns the match count or an error (n1, n2 <= 2048). */
int plvi_line_match_grid(const int* lines1, const uint8_t* desc1, int n1, int grid_cols, int grid_rows,
                         const int* cell_off, const int* cell_idx, const uint8_t* desc2, const double* directions2,
                         int n2, int win_w0, int win_w1, int win_h0, int win_h1, int libstdcxx_range_hint,
                         int* matches_12);

/* Batched device variant: pair p uses lines1 + p*cap1*4, desc1 + p*cap1*32,
 * cell_off + p*(ncell+1), cell_idx + p*idx_cap, desc2 + p*cap2*32,
 * directions2 + p*cap2*2, counts n1[p], n2[p].  Outputs matches_12
 * [n_pairs][cap1], nmatches [n_pairs]; *d_err |= 1 when a candidate set
 * exceeds 1024 lines (d_err may be NULL: no report). */
int plvi_line_match_grid_batch(int n_pairs, const int* d_lines1, const uint8_t* d_desc1, const int* d_n1, int cap1,
                               int grid_cols, int grid_rows, const int* d_cell_off, const int* d_cell_idx,
                               int idx_cap, const uint8_t* d_desc2, const double* d_directions2, const int* d_n2,
                               int cap2, int win_w0, int win_w1, int win_h0, int win_h1, int libstdcxx_range_hint,
                               int* d_matches_12, int* d_nmatches, int* d_err, void* stream);

/* LineMatcher::SearchByProjection(Frame& CurrentFrame, Frame& LastFrame,
 * const GridStructure& grid, th, angth) (src/LineMatcher.cpp:274-372; its
 * Tracking.cc:3976/3984 call sites are commented out in the reference, kept
 * for drop-in completeness).  Per last-frame line (in order): flags bit0 =
 * mvpMapLines[i] && !mvbOutlier_Line[i], bit1 = that MapLine's
 * Observations() > 0; x3dc[6] = Rcw*x3Dw+tcw of its start and end point
 * (cv::Mat float, the caller's); octave = mvKeys_Line[i].octave; the
 * MapLine descriptor.  Current frame: mvKeysUn_Line angles, descriptors,
 * blocked = mvpMapLines[i2] && Observations() > 0 on entry (NULL = none),
 * grid_Line as in plvi_line_match_grid (cell (x, y) = x * rows + y, list
 * order).  Output match [cur] = last-frame line whose MapLine the call
 * stores in mvpMapLines[i2], -1 untouched; the count of assignments. */
typedef struct plvi_line_proj_params {
  float fx, fy, cx, cy;             /* Pinhole mvParameters */
  float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  double inv_w, inv_h;              /* Frame::inv_width / inv_height (grid cells per pixel) */
  float th, angth;
  int grid_cols, grid_rows;
  int range_hint;                   /* unordered_set range-insert rule: 1 = GCC <= 10, 0 = GCC >= 11 */
  int nlevels;                      /* <= 8 */
  float scale_l[8];                 /* CurrentFrame.mvScaleFactors_l */
} plvi_line_proj_params;

int plvi_line_search_projection_batch(int n_pairs, const plvi_line_proj_params* p, const float* d_cur_angle,
                                      const uint8_t* d_cur_desc, const uint8_t* d_cur_blocked, const int* d_cur_n,
                                      int cur_cap, const int* d_cell_off, const int* d_cell_idx, int idx_cap,
                                      const uint8_t* d_last_flags, const float* d_x3dc, const int* d_last_octave,
                                      const uint8_t* d_ml_desc, const int* d_last_n, int last_cap, int* d_match,
                                      int* d_nmatches, int* d_err, void* stream);
/* d_err (may be NULL): |= 1 when a candidate set overflows, |= 2 when a last-frame
 * octave is outside [0, nlevels) (that line is skipped). */
/* One pair from host memory, synchronous (n_cur <= 2048).  Returns the
 * count or an error (PLVI_E_CAPACITY when a candidate set exceeds 1024). */
int plvi_line_search_projection(const plvi_line_proj_params* p, const float* cur_angle, const uint8_t* cur_desc,
                                const uint8_t* cur_blocked, int n_cur, const int* cell_off, const int* cell_idx,
                                const uint8_t* last_flags, const float* x3dc, const int* last_octave,
                                const uint8_t* ml_desc, int n_last, int* match);

/* ------------------------------------------------------------- Vocabulary
 * DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h), the ORB vocabulary of
 * Frame::ComputeBoW (src/Frame.cc:1115-1122) and KeyFrame::ComputeBoW
 * (src/KeyFrame.cc:111).  Node ids and word ids follow the reference's
 * loader (node i = i-th line after the header, word ids in leaf order). */
typedef struct plvi_vocabulary plvi_vocabulary;

/* loadFromTextFile (TemplatedVocabulary.h:1338-1424; System.cc:84).
 * The reference's loop also builds a node from the empty line after the
 * file's final newline; its parent, leaf flag and descriptor are never
 * assigned (the istream sentry fails), i.e. undefined behaviour.
 * emulate_tail = 0 (recommended) skips it; != 0 models one outcome: a
 * weight-0, zero-descriptor, non-word child of the root. */
int plvi_vocab_load_text(const char* path, int emulate_tail, int device, plvi_vocabulary** out);

/* Build from a node table (row i = node i+1 in file order; parent[i] < i+1):
 * the structure loadFromTextFile would produce from the same lines. */
int plvi_vocab_create(int k, int L, int scoring, int weighting, int n_nodes, const int* parent,
                      const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                      plvi_vocabulary** out);
int plvi_vocab_destroy(plvi_vocabulary* h);

/* info[6] = k, L, scoring, weighting, node count (incl. root), word count. */
int plvi_vocab_info(plvi_vocabulary* h, int* info);

/* transform(features, BowVector&, FeatureVector&, levelsup)
 * (TemplatedVocabulary.h:1126-1194) for one frame from host memory:
 * BowVector (std::map<WordId, WordValue>) as bow_word/bow_value in map order,
 * FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR fv_node[i],
 * fv_idx[fv_off[i] .. fv_off[i+1]) in map order.  Arrays hold n entries
 * (fv_off n + 1). */
int plvi_vocab_transform(plvi_vocabulary* h, const uint8_t* desc, int n, int levelsup, unsigned* bow_word,
                         double* bow_value, int* bow_n, unsigned* fv_node, int* fv_off, unsigned* fv_idx,
                         int* fv_n);

/* Per-descriptor descent (transform(feature, word_id, weight, &nid, levelsup),
 * :1217-1259): word id and the node at level L - levelsup. */
int plvi_vocab_transform_features(plvi_vocabulary* h, const uint8_t* desc, int n, int levelsup, unsigned* word,
                                  unsigned* nid);

/* Batched device variant over n_frames descriptor tables [n_frames][cap][32]
 * with counts d_count (e.g. plvi_orb_outputs): outputs [n_frames][cap]
 * (fv_off [n_frames][cap+1]) and per-frame counts.  d_feat_word/d_feat_nid
 * (nullable) receive the per-descriptor descent.  Asynchronous. */
int plvi_vocab_transform_batch(plvi_vocabulary* h, const uint8_t* d_desc, const int* d_count, int cap, int n_frames,
                               int levelsup, unsigned* d_bow_word, double* d_bow_value, int* d_bow_n,
                               unsigned* d_fv_node, int* d_fv_off, unsigned* d_fv_idx, int* d_fv_n,
                               unsigned* d_feat_word, unsigned* d_feat_nid, void* stream);

/* ----------------------------------------------------------- Undistortion
 * Frame::UndistortKeyPoints (src/Frame.cc:1124-1157), UndistortKeyLines
 * (:1159-1197) and ComputeImageBounds (:1199-1226) = cv::undistortPoints
 * (OpenCV 4.2, 5 iterations, R = I, P = K).  mDistCoef[0] == 0 copies the
 * points unchanged, as the reference does. */
typedef struct plvi_camera {
  float fx, fy, cx, cy; /* mK */
  float dist[5];        /* mDistCoef: k1, k2, p1, p2[, k3] */
  int ndist;            /* 4 or 5 */
} plvi_camera;

/* n points (x, y float pairs, device), asynchronous. */
int plvi_undistort_points(const plvi_camera* cam, const float* d_xy, int n, float* d_out, void* stream);
/* mvKeysUn of keypoint tables [n_frames][cap] (counts d_count): each
 * keypoint copied with its pt undistorted. */
int plvi_undistort_keypoints_batch(const plvi_camera* cam, const plvi_keypoint* d_kps, const int* d_count, int cap,
                                   int n_frames, plvi_keypoint* d_out, void* stream);
/* Undistorted keyline endpoints [n_frames][cap][4] = startX, startY, endX, endY. */
int plvi_undistort_keylines_batch(const plvi_camera* cam, const plvi_keyline* d_kl, const int* d_count, int cap,
                                  int n_frames, float* d_endpoints, void* stream);
/* mnMinX, mnMaxX, mnMinY, mnMaxY (synchronous). */
int plvi_image_bounds(const plvi_camera* cam, int cols, int rows, float* bounds);

/* ------------------------------------------------------ SearchByProjection
 * The steady-state frame-to-frame ORB matcher of Tracking::TrackWithMotionModel
 * (src/Tracking.cc:3957): Frame::AssignFeaturesToGrid (src/Frame.cc:644-675),
 * Frame::GetFeaturesInArea (:1006-1075) and
 * ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 * (src/ORBmatcher.cc:1962-2178, single camera: Nleft == -1). */

/* Frame grid geometry: mnMinX, mnMinY, mfGridElementWidthInv/HeightInv
 * (Frame.cc:156-157); the grid is FRAME_GRID_COLS x ROWS = 64 x 48. */
typedef struct plvi_grid_params {
  float min_x, min_y, inv_w, inv_h;
} plvi_grid_params;

/* AssignFeaturesToGrid of n_frames keypoint tables [n_frames][cap]
 * (mvKeysUn; counts d_count) as CSR: cell (ix, iy) = ix*48 + iy lists its
 * keypoints at d_cell_idx[f*cap + d_cell_off[f*3073 + cell] ...] in index
 * order (= mGrid[ix][iy]).  cap <= 8192.  Asynchronous. */
int plvi_assign_grid_batch(const plvi_keypoint* d_kps, const int* d_count, int cap, int n_frames,
                           const plvi_grid_params* gp, int* d_cell_off, int* d_cell_idx, void* stream);

typedef struct plvi_proj_params {
  float fx, fy, cx, cy;            /* Pinhole mvParameters (CameraModels/Pinhole.cpp:30-33) */
  float mbf;                       /* CurrentFrame.mbf (mvuRight check, :2041-2047) */
  float th;                        /* window radius at octave 0 (radius = th * mvScaleFactors[octave]) */
  float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  float inv_w, inv_h;              /* mfGridElementWidthInv / HeightInv */
  int forward, backward;           /* bForward / bBackward (:1982-1983; both 0 for bMono) */
  int check_orientation;           /* mbCheckOrientation */
  int nlevels;
  float scale_factors[16];         /* CurrentFrame.mvScaleFactors */
} plvi_proj_params;

/* Batched SearchByProjection over n_pairs (CurrentFrame, LastFrame) pairs.
 * Current frame p: keypoints/descriptors [p][cur_cap] (mvKeysUn, counts
 * d_cur_n), grid CSR from plvi_assign_grid_batch, blocked[i2] =
 * mvpMapPoints[i2] && Observations() > 0 on entry (NULL = none), mvuRight
 * (NULL = none).  Last frame p: [p][last_cap] x3Dc = Rcw*x3Dw + tcw of the
 * point's MapPoint (3 floats), octave (mvKeys[i].octave), angle
 * (mvKeysUn[i].angle), MapPoint descriptor (32 B), flags bit0 = has a
 * MapPoint and is not an outlier, bit1 = that MapPoint's Observations() > 0.
 * Output match [p][cur_cap]: LastFrame index whose MapPoint
 * mvpMapPoints[i2] holds on return, -2 = set to NULL by the rotation filter,
 * -1 = untouched; nmatches [p] = the return value.  cur_cap, last_cap <= 65535
 * and the LDS footprint (~19 B per current + 8 B per last keypoint + 12 KB)
 * <= 160 KB. */
int plvi_search_by_projection_batch(int n_pairs, const plvi_proj_params* p, const plvi_keypoint* d_cur_kps,
                                    const uint8_t* d_cur_desc, const int* d_cur_n, int cur_cap,
                                    const uint8_t* d_cur_blocked, const float* d_cur_uright, const int* d_cell_off,
                                    const int* d_cell_idx, const float* d_x3dc, const int* d_last_octave,
                                    const float* d_last_angle, const uint8_t* d_mp_desc, const uint8_t* d_last_flags,
                                    const int* d_last_n, int last_cap, int* d_match, int* d_nmatches, void* stream);

/* One pair from host memory, synchronous (grid built on the device).
 * Returns nmatches (>= 0) or an error. */
int plvi_search_by_projection(const plvi_proj_params* p, const plvi_keypoint* cur_kps, const uint8_t* cur_desc,
                              int n_cur, const uint8_t* cur_blocked, const float* cur_uright, const float* x3dc,
                              const int* last_octave, const float* last_angle, const uint8_t* mp_desc,
                              const uint8_t* last_flags, int n_last, int* match);

/* The same search with a two-camera CurrentFrame (CurrentFrame.Nleft != -1,
 * src/ORBmatcher.cc:1985-2153).  kb8 = KannalaBrandt8 k1..k4 of
 * CurrentFrame.mpCamera (fx, fy, cx, cy from p; NULL = Pinhole).  Left:
 * mvKeys [p][cap] (counts d_n), descriptor rows 0..Nleft-1, blocked, mGrid
 * (plvi_assign_grid_batch over the left keypoints); right: mvKeysRight
 * [p][cap_r], rows Nleft.., blocked of mvpMapPoints[Nleft + idx], mGridRight
 * (the grid kernel over the right keypoints).  LastFrame point i: x3Dc, x3Dr
 * = mTrl * x3Dc (the caller's cv::Mat products), octave (mvKeys[i] or
 * mvKeysRight[i - Nleft] of LastFrame), angle (mvKeysUn / mvKeys /
 * mvKeysRight as :2067-2069), descriptor, flags as above.  A point is
 * searched in the right image only when its left pass did not end early
 * (behind the camera, outside mnMin/MaxX/Y, empty window: :2000-2026).
 * Outputs match [p][cap] / match_r [p][cap_r] (-2 = NULL by the rotation
 * filter, which sees both images' matches in one histogram), nmatches [p].
 * A searched point whose octave is outside [0, nlevels) gets no candidate in
 * either image (the reference would index mvScaleFactors out of range).
 * p->mbf is unused.  Asynchronous on `stream`. */
int plvi_search_by_projection_stereo_batch(int n_pairs, const plvi_proj_params* p, const float* kb8,
                                           const plvi_keypoint* d_kps, const uint8_t* d_desc, const int* d_n, int cap,
                                           const uint8_t* d_blocked, const int* d_cell_off, const int* d_cell_idx,
                                           const plvi_keypoint* d_kps_r, const uint8_t* d_desc_r, const int* d_n_r,
                                           int cap_r, const uint8_t* d_blocked_r, const int* d_cell_off_r,
                                           const int* d_cell_idx_r, const float* d_x3dc, const float* d_x3dr,
                                           const int* d_last_octave, const float* d_last_angle,
                                           const uint8_t* d_mp_desc, const uint8_t* d_last_flags, const int* d_last_n,
                                           int last_cap, int* d_match, int* d_match_r, int* d_nmatches, void* stream);

/* One pair from host memory, synchronous; the same contract as the batch
 * (an octave outside [0, nlevels): no candidate).  Returns nmatches or an
 * error. */
int plvi_search_by_projection_stereo(const plvi_proj_params* p, const float* kb8, const plvi_keypoint* kps,
                                     const uint8_t* desc, int n, const uint8_t* blocked, const plvi_keypoint* kps_r,
                                     const uint8_t* desc_r, int n_r, const uint8_t* blocked_r, const float* x3dc,
                                     const float* x3dr, const int* last_octave, const float* last_angle,
                                     const uint8_t* mp_desc, const uint8_t* last_flags, int n_last, int* match,
                                     int* match_r);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
 * const set<MapPoint*>& sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:2180-2300):
 * the relocalization guided search of Tracking::Relocalization
 * (src/Tracking.cc:5857 th 10 / ORBdist 100, :5871 th 3 / ORBdist 64, with
 * ORBmatcher(0.9, true)), single camera.  The MapPoint reads stay with the
 * caller (they take the MapPoint mutexes): per KF MapPoint i, in
 * pKF->GetMapPointMatches() order,
 *   flags bit0 = pMP && !pMP->isBad() && !sAlreadyFound.count(pMP);
 *   x3dc [3]   = Rcw*x3Dw + tcw (cv::Mat float gemm);
 *   dist [3]   = { dist3D = cv::norm(x3Dw - Ow), GetMinDistanceInvariance(),
 *                  GetMaxDistanceInvariance() };
 *   level      = pMP->PredictScale(dist3D, &CurrentFrame);
 *   angle      = pKF->mvKeysUn[i].angle;  desc = pMP->GetDescriptor().
 * The device does the rest: Pinhole::project, the bounds and distance tests,
 * GetFeaturesInArea(u, v, th*mvScaleFactors[level], level-1, level+1), the
 * best candidate among keypoints whose mvpMapPoints[i2] is NULL (those
 * assigned earlier in the same call included), bestDist <= ORBdist, and the
 * rotation-histogram filter. */
typedef struct plvi_reloc_params {
  float fx, fy, cx, cy;             /* Pinhole mvParameters */
  float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  float inv_w, inv_h;               /* mfGridElementWidthInv / HeightInv */
  float th;                         /* window radius at level 0 */
  int orb_dist;                     /* ORBdist (< 256: at 256 an empty search would index mvpMapPoints[-1]) */
  int check_orientation;            /* mbCheckOrientation */
  int nlevels;                      /* CurrentFrame.mnScaleLevels (levels outside [0, nlevels) get no candidate) */
  float scale_factors[16];          /* CurrentFrame.mvScaleFactors */
} plvi_reloc_params;

/* Batched over n_pairs (CurrentFrame, KeyFrame) pairs.  Current frame p:
 * keypoints/descriptors [p][cur_cap] (mvKeysUn, counts d_cur_n), grid CSR from
 * plvi_assign_grid_batch, blocked[i2] = mvpMapPoints[i2] != NULL on entry
 * (NULL = none).  KeyFrame p: [p][kf_cap] flags, x3dc [3], dist [3], level,
 * angle, desc [32] as above (counts d_kf_n).  Output match [p][cur_cap]: KF
 * MapPoint index stored in mvpMapPoints[i2] by the call, -2 = set to NULL by
 * the rotation filter, -1 = untouched; nmatches [p] = the return value.
 * cur_cap, kf_cap <= 65535 and ~19 B per current + 8 B per KF point + 12 KB of
 * LDS <= 160 KB.  Asynchronous on `stream`. */
int plvi_search_reloc_batch(int n_pairs, const plvi_reloc_params* p, const plvi_keypoint* d_cur_kps,
                            const uint8_t* d_cur_desc, const int* d_cur_n, int cur_cap, const uint8_t* d_cur_blocked,
                            const int* d_cell_off, const int* d_cell_idx, const uint8_t* d_kf_flags,
                            const float* d_x3dc, const float* d_dist, const int* d_level, const float* d_kf_angle,
                            const uint8_t* d_mp_desc, const int* d_kf_n, int kf_cap, int* d_match, int* d_nmatches,
                            void* stream);

/* One pair from host memory, synchronous (grid built on the device).
 * Returns nmatches (>= 0) or an error. */
int plvi_search_reloc(const plvi_reloc_params* p, const plvi_keypoint* cur_kps, const uint8_t* cur_desc, int n_cur,
                      const uint8_t* cur_blocked, const uint8_t* kf_flags, const float* x3dc, const float* dist,
                      const int* level, const float* kf_angle, const uint8_t* mp_desc, int n_kf, int* match);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&
 * vpMapPoints, th, bFarPoints, thFarPoints) (src/ORBmatcher.cc:44-145,
 * F.Nleft == -1, RadiusByViewingCos :216-222): the local-map search of
 * Tracking::SearchLocalPoints (src/Tracking.cc:5119/5211). */
typedef struct plvi_local_params {
  float min_x, min_y, inv_w, inv_h; /* F.mnMinX, mnMinY, mfGridElementWidthInv / HeightInv */
  float th;                         /* th (the radius is scaled by th when th != 1) */
  float nnratio;                    /* ORBmatcher(nnratio): 0.8 in SearchLocalPoints */
  int nlevels;
  float scale_factors[16];          /* F.mvScaleFactors */
} plvi_local_params;

/* Batched over n_frames frames: frame f's keypoints (mvKeysUn) /
 * descriptors [f][cap] (counts d_n), grid CSR from plvi_assign_grid_batch,
 * blocked[idx] = mvpMapPoints[idx] && Observations() > 0 on entry (NULL =
 * none), mvuRight (NULL = none); its MapPoints [f][mp_cap] (counts d_mp_n,
 * vector order): flags bit0 = searched (mbTrackInView && not far &&
 * !isBad()), bit1 = Observations() > 0; proj [4] = mTrackProjX,
 * mTrackProjY, mTrackProjXR, mTrackViewCos; level = mnTrackScaleLevel;
 * GetDescriptor() (32 B).  Output match [f][cap] = the MapPoint index
 * stored in F.mvpMapPoints[idx] by the call, or -1; nmatches [f] = the
 * return value.  A MapPoint whose level is outside [0, nlevels) gets no
 * candidate.  cap <= 65535 and ~17 B per keypoint + 8 B per MapPoint +
 * 12 KB of LDS <= 160 KB. */
int plvi_search_local_batch(int n_frames, const plvi_local_params* p, const plvi_keypoint* d_kps, const uint8_t* d_desc,
                            const int* d_n, int cap, const uint8_t* d_blocked, const float* d_uright,
                            const int* d_cell_off, const int* d_cell_idx, const uint8_t* d_mp_flags,
                            const float* d_mp_proj, const int* d_mp_level, const uint8_t* d_mp_desc, const int* d_mp_n,
                            int mp_cap, int* d_match, int* d_nmatches, void* stream);

/* One frame from host memory, synchronous.  Returns nmatches or an error. */
int plvi_search_local(const plvi_local_params* p, const plvi_keypoint* kps, const uint8_t* desc, int n,
                      const uint8_t* blocked, const float* uright, const uint8_t* mp_flags, const float* mp_proj,
                      const int* mp_level, const uint8_t* mp_desc, int n_mp, int* match);

/* The same search on a two-camera Frame (F.Nleft != -1, src/ORBmatcher.cc:
 * 44-214; replaces the reference's loop for KannalaBrandt8 stereo rigs).
 * Left side: mvKeys [f][cap] (counts d_n) with their descriptors (rows
 * 0..Nleft-1 of mDescriptors), blocked (mvpMapPoints[idx] && Observations()
 * > 0), mvLeftToRightMatch (NULL = all -1) and the left grid (mGrid,
 * plvi_assign_grid_batch over the left keypoints); right side: mvKeysRight
 * [f][cap_r] (counts d_n_r), descriptors rows Nleft.., blocked of
 * mvpMapPoints[Nleft + idx], mvRightToLeftMatch and mGridRight (the grid
 * kernel over the right keypoints: right-relative indices).  MapPoints:
 * flags bit0 = searched left (mbTrackInView && not far && !isBad()), bit1 =
 * Observations() > 0, bit2 = searched right (mbTrackInViewR && not far &&
 * !isBad()); proj [4] = mTrackProjX, mTrackProjY, (unused), mTrackViewCos;
 * level = mnTrackScaleLevel; proj_r [4] = mTrackProjXR, mTrackProjYR,
 * (unused), mTrackViewCosR; level_r = mnTrackScaleLevelR (-1: no right
 * search).  Outputs match [f][cap] / match_r [f][cap_r] = the MapPoint
 * index stored in mvpMapPoints[idx] / mvpMapPoints[Nleft + idx] by the
 * call, or -1; nmatches [f] = the return value.  Asynchronous on `stream`. */
int plvi_search_local_stereo_batch(int n_frames, const plvi_local_params* p, const plvi_keypoint* d_kps,
                                   const uint8_t* d_desc, const int* d_n, int cap, const uint8_t* d_blocked,
                                   const int* d_l2r, const int* d_cell_off, const int* d_cell_idx,
                                   const plvi_keypoint* d_kps_r, const uint8_t* d_desc_r, const int* d_n_r, int cap_r,
                                   const uint8_t* d_blocked_r, const int* d_r2l, const int* d_cell_off_r,
                                   const int* d_cell_idx_r, const uint8_t* d_mp_flags, const float* d_mp_proj,
                                   const int* d_mp_level, const float* d_mp_proj_r, const int* d_mp_level_r,
                                   const uint8_t* d_mp_desc, const int* d_mp_n, int mp_cap, int* d_match,
                                   int* d_match_r, int* d_nmatches, void* stream);

/* One two-camera frame from host memory, synchronous.  Returns nmatches or
 * an error. */
int plvi_search_local_stereo(const plvi_local_params* p, const plvi_keypoint* kps, const uint8_t* desc, int n,
                             const uint8_t* blocked, const int* l2r, const plvi_keypoint* kps_r, const uint8_t* desc_r,
                             int n_r, const uint8_t* blocked_r, const int* r2l, const uint8_t* mp_flags,
                             const float* mp_proj, const int* mp_level, const float* mp_proj_r, const int* mp_level_r,
                             const uint8_t* mp_desc, int n_mp, int* match, int* match_r);

/* --------------------------------------------------------------- Frustum
 * The local-map visibility test of Tracking::SearchLocalPoints /
 * SearchLocalPointsAndLines (src/Tracking.cc:5074-5092, :5166-5184,
 * :5219-5234): Frame::isInFrustum (src/Frame.cc:758-835, Nleft == -1;
 * :836-846 + isInFrustumChecks :1751-1824, Nleft != -1), Frame::isInFrustum_l
 * (:849-933), MapPoint::PredictScale(dist, Frame*) (src/MapPoint.cc:531-546),
 * Get{Min,Max}DistanceInvariance (MapPoint.cc:502-512, MapLine.cc:384-394).
 * The outputs are the MapPoint fields the local search reads, in the layout
 * of plvi_search_local_batch / plvi_search_local_stereo_batch, so the two run
 * back to back on the device.
 *
 * One camera of a frame: the world->camera pose of the product Pc = R*P + t
 * and the centre O of the distance test.  Left / one-camera frames: R = mRcw,
 * t = mtcw, O = mOw, the camera mpCamera.  Right camera of a two-camera frame:
 * R = Rrl*mRcw, t = Rrl*mtcw + trl, O = mRwc*tlr + mOw (Frame.cc:1757-1761,
 * per frame, the caller's cv::Mat products), the camera mpCamera2. */
typedef struct plvi_frustum_camera {
  float R[9]; /* row-major */
  float t[3];
  float O[3];
  float fx, fy, cx, cy; /* Pinhole / KannalaBrandt8 mvParameters[0..3]; lines: Frame::fx, fy, cx, cy */
  float kb[4];          /* KannalaBrandt8 k1..k4 (mvParameters[4..7]) */
  int model;            /* 0 = Pinhole, 1 = KannalaBrandt8 */
} plvi_frustum_camera;

typedef struct plvi_frustum_params {
  plvi_frustum_camera cam[2];       /* cam[1] only with two_camera */
  int two_camera;                   /* F.Nleft != -1 */
  float mbf;                        /* Frame::mbf (mTrackProjXR of a one-camera frame) */
  float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
  float view_cos_limit;             /* 0.5 in SearchLocalPoints */
  int far_points;                   /* mpLocalMapper->mbFarPoints */
  float far_th;                     /* mpLocalMapper->mThFarPoints */
  int nlevels;                      /* mnScaleLevels (1..16) */
  float log_scale_factor;           /* mfLogScaleFactor */
  float level_ratio[16];            /* filled by plvi_frustum_params_init */
  unsigned compat;                  /* PLVI_COMPAT_GEMM_FMA */
} plvi_frustum_params;

/* PredictScale as a table: level_ratio[n] = the least float ratio =
 * mfMaxDistance/dist with ceil(logf(ratio)/mfLogScaleFactor) >= n (host glibc
 * logf, as MapPoint.cc.o calls it); +inf when none.  Call once per
 * (nlevels, log_scale_factor) before uploading the params.  PLVI_E_BADARG for
 * nlevels outside 1..16 or a negative / NaN log_scale_factor. */
int plvi_frustum_params_init(plvi_frustum_params* p);

/* Output flags of plvi_frustum_points_batch. */
enum {
  PLVI_FRUSTUM_SEARCH = 1,    /* searched by SearchByProjection (left): in view, not far (== local bit0) */
  PLVI_FRUSTUM_OBS = 2,       /* Observations() > 0, copied from the input (== local bit1) */
  PLVI_FRUSTUM_SEARCH_R = 4,  /* two-camera: searched right (== local-stereo bit2) */
  PLVI_FRUSTUM_VISIBLE = 8,   /* isInFrustum returned true: IncreaseVisible, nToMatch */
  PLVI_FRUSTUM_TRACK = 16,    /* mbTrackInView after the call: mmProjectPoints[mnId] = (ProjX, ProjY) */
};

/* Per frame f (d_params[f] on the device), its local MapPoints [f][cap] in
 * mvpLocalMapPoints order (counts d_n): pos [3] = GetWorldPos(), normal [3] =
 * GetNormal(), dist [2] = {mfMinDistance, mfMaxDistance}, in_flags bit0 =
 * the loop reaches isInFrustum (mnLastFrameSeen != mnId && !isBad()), bit1 =
 * Observations() > 0.  Outputs, for evaluated MapPoints only (others keep the
 * buffers' contents, flags 0 apart from OBS): proj [4] = {mTrackProjX,
 * mTrackProjY, mTrackProjXR, mTrackViewCos}, level = mnTrackScaleLevel, depth
 * = mTrackDepth (in/out: a two-camera far test reads the entry value when the
 * left test fails); two-camera frames: proj[2] untouched, proj_r [4] =
 * {mTrackProjXR, mTrackProjYR, -, mTrackViewCosR}, level_r =
 * mnTrackScaleLevelR (-1 = not in view).  Fields the reference leaves stale
 * are left as they were.  nvisible [f] = nToMatch.  proj_r / level_r may be
 * NULL for one-camera batches, nvisible may be NULL.  Asynchronous. */
int plvi_frustum_points_batch(int n_frames, const plvi_frustum_params* d_params, const float* d_pos,
                              const float* d_normal, const float* d_dist, const uint8_t* d_in_flags, const int* d_n,
                              int cap, uint8_t* d_flags, float* d_proj, int* d_level, float* d_proj_r, int* d_level_r,
                              float* d_depth, int* d_nvisible, void* stream);

/* One frame from host memory, synchronous.  Returns nToMatch or an error. */
int plvi_frustum_points(const plvi_frustum_params* p, const float* pos, const float* normal, const float* dist,
                        const uint8_t* in_flags, int n, uint8_t* flags, float* proj, int* level, float* proj_r,
                        int* level_r, float* depth);

/* isInFrustum_l over frame f's local MapLines [f][cap] (mvpLocalMapLines
 * order, counts d_n): sep [6] = GetWorldPos() (double), normal [3] =
 * GetNormal(), dist [2] = {mfMinDistance, mfMaxDistance}, in_flags bit0 =
 * evaluated (mnLastFrameSeen != mnId && !isBad()), desc [32] =
 * GetDescriptor() (NULL: no gather).  Outputs: inview = mbTrackInView (0 for
 * lines not evaluated), proj [4] = {mTrackProjsX, mTrackProjsY, mTrackProjeX,
 * mTrackProjeY} (each pair written once its endpoint passes, as the
 * reference does), angle = mnTrackangle (in view only); the order-preserving
 * list mvpLocalMapLines_InFrustum as local indices compact [f][cap] (count
 * ncompact [f] = nToMatch) and their descriptors compact_desc [f][cap][32],
 * the desc1 of LineMatcher::match (plvi_line_match_batch).  Asynchronous. */
int plvi_frustum_lines_batch(int n_frames, const plvi_frustum_params* d_params, const double* d_sep,
                             const float* d_normal, const float* d_dist, const uint8_t* d_in_flags,
                             const uint8_t* d_desc, const int* d_n, int cap, uint8_t* d_inview, float* d_proj,
                             double* d_angle, int* d_compact, uint8_t* d_compact_desc, int* d_ncompact, void* stream);

/* One frame from host memory, synchronous.  Returns nToMatch or an error. */
int plvi_frustum_lines(const plvi_frustum_params* p, const double* sep, const float* normal, const float* dist,
                       const uint8_t* in_flags, const uint8_t* desc, int n, uint8_t* inview, float* proj,
                       double* angle, int* compact, uint8_t* compact_desc);

/* The orientation / position filter after LineMatcher::match in
 * SearchLocalPointsAndLines (src/Tracking.cc:5244-5292).  Frame f: matches_12
 * [f][cap] over its ncompact [f] in-frustum lines (in/out: rejected entries
 * set to -1, as the reference does), compact / proj / angle from
 * plvi_frustum_lines_batch, the frame's mvKeysUn_Line [f][kl_cap] (counts
 * d_nkl), blocked [f][kl_cap] = mvpMapLines[i2] && Observations() > 0 on
 * entry (NULL = none).  Output assign [f][kl_cap] = the local MapLine index
 * stored in mvpMapLines[i2] by the loop, or -1; nassigned [f] = their count.
 * The bounds for deltaWidth / deltaHeight come from d_params[f]. */
int plvi_local_lines_filter_batch(int n_frames, const plvi_frustum_params* d_params, int* d_matches_12,
                                  const int* d_ncompact, const int* d_compact, int cap, const float* d_proj,
                                  const double* d_angle, const plvi_keyline* d_kl, const int* d_nkl, int kl_cap,
                                  const uint8_t* d_blocked, int* d_assign, int* d_nassigned, void* stream);

/* ---------------------------------------------------------------- Stereo
 * Rectified stereo of the stereo Frame constructors (src/Frame.cc:95-140,
 * :225-300). */

/* Frame::ComputeStereoMatches (src/Frame.cc:1228-1406) for n_frames pairs
 * extracted by two ORB handles of the same geometry (mpORBextractorLeft /
 * Right, vLappingArea {0,0}): keypoints, descriptors and mvImagePyramid are
 * read on the device.  mb / mbf: Frame::mb, mbf.  Outputs mvuRight /
 * mvDepth [n_frames][cap] (cap of plvi_orb_outputs, -1 = no depth),
 * d_nstereo [n_frames] = left keypoints with a depth; *d_err |= 1 when a
 * right keypoint's row band leaves the image (the reference indexes
 * vRowIndices out of range), |= 2 when an SAD window leaves its level (the
 * reference's rowRange/colRange assert).  Asynchronous on `stream`. */
int plvi_stereo_match_batch(plvi_orb_extractor* left, plvi_orb_extractor* right, int n_frames, float mb, float mbf,
                            float* d_uright, float* d_depth, int* d_nstereo, int* d_err, void* stream);

/* One pair from host memory, synchronous.  Pyramids: level l of each side
 * at pyr + lvl_off[l], lvl_w[l] x lvl_h[l] (row stride lvl_w[l]); scale /
 * inv_scale = mvScaleFactors / mvInvScaleFactors.  Returns the number of
 * left keypoints with a depth, or an error (PLVI_E_OVERFLOW for the
 * reference's out-of-range cases above). */
int plvi_stereo_match(const plvi_keypoint* kpsL, const uint8_t* descL, int nL, const plvi_keypoint* kpsR,
                      const uint8_t* descR, int nR, int nlevels, const float* scale, const float* inv_scale,
                      const uint8_t* pyrL, const uint8_t* pyrR, const long long* lvl_off, const int* lvl_w,
                      const int* lvl_h, float mb, float mbf, float* uright, float* depth);

/* Frame::ComputeStereoMatches_Lines (src/Frame.cc:1408-1492): GridStructure
 * of the right lines (getLineCoords, src/gridStructure.cpp:32-40), the
 * line_2d coordinates and directions, LineMatcher::matchGrid with the
 * stereo window {width (7,0), height (2,2)}, then the endpoint disparities
 * (lineSegmentOverlapStereo :1494-1529, filterLineSegmentDisparity
 * :1531-1542) and mvle_l from mvKeysUn_Line (d_klUn; NULL = the left
 * keylines).  Per pair p: keylines/descriptors at p*cap, counts n[p].
 * Outputs matches_12 [n][capL], mvDisparity_l / mvDepth_l [n][capL][2]
 * floats (-1 = none), mvle_l [n][capL][3] doubles (0 when either side has
 * no lines, as the reference returns before computing it), d_nstereo [n].
 * d_scratch: plvi_stereo_lines_scratch_bytes(n, capL, capR, idx_cap) bytes;
 * idx_cap bounds the grid entries of one frame (*d_err |= 4 if exceeded).
 * Asynchronous on `stream`. */
size_t plvi_stereo_lines_scratch_bytes(int n_frames, int capL, int capR, int idx_cap);
int plvi_stereo_lines_batch(int n_frames, const plvi_keyline* d_klL, const uint8_t* d_descL, const int* d_nL, int capL,
                            const plvi_keyline* d_klR, const uint8_t* d_descR, const int* d_nR, int capR,
                            const plvi_keyline* d_klUn, int width, int height, float mbf, int libstdcxx_range_hint,
                            int idx_cap, void* d_scratch, size_t scratch_bytes, int* d_matches_12, float* d_disparity,
                            float* d_depth, double* d_le, int* d_nstereo, int* d_err, void* stream);

/* One pair from host memory, synchronous (n <= 2048 lines per side).
 * Returns the number of lines with a depth, or an error. */
int plvi_stereo_lines(const plvi_keyline* klL, const uint8_t* descL, int nL, const plvi_keyline* klR,
                      const uint8_t* descR, int nR, const plvi_keyline* klUn, int width, int height, float mbf,
                      int libstdcxx_range_hint, int* matches_12, float* disparity, float* depth, double* le);

/* ------------------------------------------------------------ Frame level
 * Frame::Frame's extraction (src/Frame.cc:537-641, ExtractORB/ExtractLine
 * :677-692): the ORB and line extractors on the same batch of frames, run
 * as one schedule (LSD prep, then region growing concurrent with the ORB
 * pipeline and the LBD Sobel pyramid on the handles' own streams).
 * Asynchronous with respect to `stream`, which it joins at the end; the
 * results are read with plvi_orb_outputs / plvi_lines_outputs. */
int plvi_frame_extract_batch(plvi_orb_extractor* orb, plvi_line_extractor* lines, const uint8_t* d_frames,
                             int n_frames, size_t frame_stride, size_t row_stride, int lap0, int lap1, void* stream);

/* plvi_frame_extract_batch followed by the step's matching of every frame t
 * in the batch against frame t-1: the ORB kNN-2 (plvi_hamming_knn2_batch of
 * descriptor rows t vs t-1: outputs [n_frames-1][orb cap]) issued on the
 * schedule's ORB stream as soon as the ORB extraction is done, and
 * LineMatcher::match (plvi_line_match_batch, nnr, scratch as there: outputs
 * [n_frames-1][line cap]) on the line path's stream right after the LBD
 * descriptors -- no join of the schedule's streams in between.  Joins
 * `stream` at the end.  n_frames >= 2. */
int plvi_frame_extract_match_batch(plvi_orb_extractor* orb, plvi_line_extractor* lines, const uint8_t* d_frames,
                                   int n_frames, size_t frame_stride, size_t row_stride, int lap0, int lap1,
                                   int* d_idx0, int* d_d0, int* d_idx1, int* d_d1, float nnr, int* d_line_scratch,
                                   int* d_line_matches, int* d_line_nmatch, void* stream);

/* The event the last plvi_frame_extract_batch on `lines` recorded once its
 * ORB extraction was complete (a hipEvent_t owned by the handle): work on the
 * ORB tables -- kNN-2 against the previous frame -- can wait on it
 * (plvi_stream_wait_event) and overlap the rest of the line path instead of
 * waiting for the whole frame.  After plvi_frame_extract_match_batch the same
 * event is recorded after the ORB kNN-2 as well (it then covers extraction
 * AND d_idx0/d_d0/d_idx1/d_d1).  The handle re-records it on its next
 * extract call: issue every wait on it before the next extract call on the
 * same handle, or the wait refers to the newer batch. */
int plvi_frame_orb_event(plvi_line_extractor* lines, void** event);

/* ------------------------------------------------------------ initialization
 * The monocular initializer's matchers, called on every frame until
 * Tracking::MonocularInitialization succeeds (src/Tracking.cc:3111-3113). */

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12,
 * windowSize) (src/ORBmatcher.cc:705-814). */
typedef struct plvi_init_params {
  float min_x, min_y, inv_w, inv_h; /* F2.mnMinX, mnMinY, mfGridElementWidthInv / HeightInv */
  int window;                       /* windowSize (100 in MonocularInitialization) */
  float nnratio;                    /* ORBmatcher(0.9, true): mfNNratio */
  int check_orientation;            /* mbCheckOrientation */
} plvi_init_params;

/* Batched over n_pairs (F1 = mInitialFrame, F2 = mCurrentFrame) pairs.
 * F1 p: keypoints (mvKeysUn) / descriptors [p][cap1] (counts d_n1) and
 * vbPrevMatched as float2 [p][cap1] (in/out: matched entries become
 * F2.mvKeysUn[vnMatches12[i1]].pt, as the reference updates them); F2 p:
 * keypoints / descriptors [p][cap2] (counts d_n2) and the grid CSR from
 * plvi_assign_grid_batch over the same keypoints.  Output vnMatches12
 * [p][cap1] (first n1 entries) and nmatches [p].  cap1, cap2 <= 65535 and
 * ~24 B per F1 + ~19 B per F2 keypoint + 12 KB of LDS <= 160 KB.
 * Replaces ORBmatcher.h:71 (SearchForInitialization). */
int plvi_search_for_initialization_batch(int n_pairs, const plvi_init_params* p, const plvi_keypoint* d_kps1,
                                         const uint8_t* d_desc1, const int* d_n1, int cap1, float* d_prev_matched,
                                         const plvi_keypoint* d_kps2, const uint8_t* d_desc2, const int* d_n2,
                                         int cap2, const int* d_cell_off, const int* d_cell_idx, int* d_matches12,
                                         int* d_nmatches, void* stream);

/* LineMatcher::SerachForInitialize(InitialFrame, CurrentFrame, LineMatches)
 * (src/LineMatcher.cpp:113-139) with Frame::lineDescriptorMAD
 * (src/Frame.cc:1089-1112): knnMatch(k=2) of the initial frame's LBD
 * descriptors [p][cap1] (counts d_n1) against the current frame's [p][cap2],
 * then the pairs whose d1 - d0 exceeds 0.5 * nn12_mad.  Output LineMatches
 * as int2 (query, train) [p][cap1] in query order, their count [p], and
 * (nullable) {nn_mad, nn12_mad} as double [p][2].  d_scratch holds
 * 4 * n_pairs * cap1 ints.  The reference reads lmatches[0] and [i][1]:
 * with no query lines or fewer than 2 train lines it is undefined; here the
 * pair gets 0 matches.  Replaces LineMatcher.h:95 (SerachForInitialize). */
int plvi_line_search_init_batch(const uint8_t* d_desc1, const int* d_n1, int cap1, const uint8_t* d_desc2,
                                const int* d_n2, int cap2, int n_pairs, int* d_scratch, int* d_pairs, int* d_npairs,
                                double* d_mad, void* stream);

/* The stereo-line Frame ctor (src/Frame.cc:200-249: ExtractORB left || right,
 * ExtractLine left || right): both sides' ORB + line extraction of a batch of
 * rectified pairs as two concurrent frame schedules (the right one forked
 * from `stream` onto lines_right's own stream and joined back).  Asynchronous
 * on `stream`; each handle keeps its side's results (plvi_orb_outputs /
 * plvi_lines_outputs), which plvi_stereo_match_batch and
 * plvi_stereo_lines_batch then read on the same stream.  Left and right
 * handles must be distinct. */
int plvi_stereo_frame_extract_batch(plvi_orb_extractor* orb_left, plvi_orb_extractor* orb_right,
                                    plvi_line_extractor* lines_left, plvi_line_extractor* lines_right,
                                    const uint8_t* d_left, const uint8_t* d_right, int n_frames, size_t frame_stride,
                                    size_t row_stride, int lap0, int lap1, void* stream);

/* Device memory helpers for bindings that have no HIP runtime of their own
 * (ctypes, JNI): thin wrappers over hipMalloc/hipFree/hipMemcpy on the
 * current device.  kind: 1 = host->device, 2 = device->host, 3 = d->d. */
int plvi_device_malloc(void** ptr, size_t bytes);
int plvi_device_free(void* ptr);
int plvi_memcpy(void* dst, const void* src, size_t bytes, int kind);
/* Same, asynchronous on `stream` (hipStream_t). */
int plvi_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream);
int plvi_device_synchronize(void);
/* A non-blocking HIP stream (hipStreamCreateWithFlags(hipStreamNonBlocking))
 * for bindings without a HIP runtime of their own; destroy / synchronize. */
int plvi_stream_create(void** stream);
int plvi_stream_destroy(void* stream);
int plvi_stream_synchronize(void* stream);
/* Events for the same bindings (hipEventCreateWithFlags(hipEventDisableTiming),
 * hipEventRecord, hipStreamWaitEvent, hipEventDestroy). */
int plvi_event_create(void** event);
int plvi_event_record(void* event, void* stream);
int plvi_stream_wait_event(void* stream, void* event);
int plvi_event_destroy(void* event);

/* HIP graphs (no reference counterpart: a runtime facility of this
 * library).  plvi_graph_capture_begin starts capturing `stream` (a created
 * stream, not the null stream); every plvi_* call issued on it until
 * plvi_graph_capture_end is recorded, not run, including the work the
 * extractors fork to their own streams.  The captured step is instantiated
 * into *graph_exec and replayed by plvi_graph_launch with the same device
 * pointers and parameters; plvi_graph_destroy frees it.  The multi-stream
 * frame schedule (plvi_frame_extract_batch) needs HIP runtime >= 7.2 to be
 * captured (the 7.0 runtime crashes in hipStreamEndCapture on its
 * fork/join): on an older runtime it returns PLVI_E_CAPTURE while capturing. */
int plvi_graph_capture_begin(void* stream);
int plvi_graph_capture_end(void* stream, void** graph_exec);
int plvi_graph_launch(void* graph_exec, void* stream);
int plvi_graph_destroy(void* graph_exec);

/* Device/library information for diagnostics. */
const char* plvi_version(void);
int plvi_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* PLVI_FRONTEND_H */
