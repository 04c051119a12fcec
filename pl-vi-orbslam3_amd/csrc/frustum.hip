// frustum.hip — the local-map visibility test on the device:
//   Frame::isInFrustum(pMP, viewingCosLimit)   src/Frame.cc:758-835 (Nleft == -1)
//     two-camera frames: :836-846 + isInFrustumChecks :1751-1824
//   Frame::isInFrustum_l(pML, viewingCosLimit) src/Frame.cc:849-933
//   MapPoint::PredictScale(dist, Frame*)       src/MapPoint.cc:531-546
//   Get{Min,Max}DistanceInvariance             src/MapPoint.cc:502-512, src/MapLine.cc:384-394
//   the orientation / position filter after LineMatcher::match
//                                              src/Tracking.cc:5244-5292
// as Tracking::SearchLocalPoints / SearchLocalPointsAndLines call them
// (src/Tracking.cc:5074-5092, :5166-5184, :5219-5234).  The outputs are the
// MapPoint / MapLine fields the local searches read, in the layout
// search_local_kernel / search_local2_kernel (proj.hip) and
// plvi_line_match_batch (grid_match.hip) take, so the whole local-map step
// stays on the device.
//
// Arithmetic as the reference objects do it (Frame.cc.o, MapPoint.cc.o,
// pinned by tests/test_ref_objects.py): the pose product is OpenCV's
// small-matrix gemm (float products and sums, one double add of t, parity
// unpinned beyond that: PLVI_COMPAT_GEMM_FMA picks the AVX2-dispatched
// contraction); cv::norm / Mat::dot of 3-vectors accumulate the exact float
// squares / products in double; mTrackProjXR = fma(-mbf, invz, u) and the
// line endpoints u = fma(fx*PcX, invz, cx) are the fused sites of Frame.cc.o.
// PredictScale's glibc logf is a per-frame threshold table
// (plvi_frustum_params_init on the host): level = #{n : ratio >=
// level_ratio[n]}, with cvttss2si's INT_MIN -> 0 for an infinite ratio.
//
// Work: one thread per MapPoint (2-D grid: chunk x frame), ~62 B of HBM
// traffic each; lines one workgroup per frame for the order-preserving
// compaction of mvpLocalMapLines_InFrustum (ballot + wave prefix).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "plvi_common.h"
#include "plvi_math.h"

namespace plvi {

namespace {

// cv::gemm(R, P, 1, t, 1) for R 3x3, P / t 3x1 float (MatExpr R*P + t).
__device__ __forceinline__ float pose_row(const float* R, float px, float py, float pz, float t, bool fma_form) {
    const float s = fma_form ? rfmaf(R[2], pz, rfmaf(R[0], px, R[1] * py)) : (R[0] * px + R[1] * py) + R[2] * pz;
    return (float)((double)s + (double)t);
}

// cv::norm(v) (NORM_L2, 3x1 float): exact float squares summed in double.
__device__ __forceinline__ double cv_norm3(float a, float b, float c) {
    double s = 0.0;
    s += (double)a * a;
    s += (double)b * b;
    s += (double)c * c;
    return __builtin_sqrt(s);
}

// Mat::dot (3x1 float): exact products summed in double.
__device__ __forceinline__ double cv_dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    double r = 0.0;
    r += (double)a0 * b0;
    r += (double)a1 * b1;
    r += (double)a2 * b2;
    return r;
}

// GeometricCamera::project(const cv::Mat&): Pinhole (Pinhole.cpp:30-39) or
// KannalaBrandt8 (KannalaBrandt8.cpp:28-50; its seven fused multiply-adds).
__device__ __forceinline__ void cam_project(const plvi_frustum_camera& c, float x, float y, float z, float& u,
                                            float& v) {
    if (!c.model) {
        u = c.fx * x / z + c.cx;
        v = c.fy * y / z + c.cy;
        return;
    }
    const float x2_plus_y2 = rfmaf(x, x, y * y);
    const float theta = plvi_atan2f(__builtin_sqrtf(x2_plus_y2), z);
    const float psi = plvi_atan2f(y, x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = rfmaf(c.kb[3], theta9, rfmaf(c.kb[2], theta7, rfmaf(c.kb[1], theta5, rfmaf(c.kb[0], theta3, theta))));
    u = rfmaf(c.fx * r, plvi_cosf(psi), c.cx);
    v = rfmaf(c.fy * r, plvi_sinf(psi), c.cy);
}

// MapPoint::PredictScale(dist, Frame*) from the threshold table.
__device__ __forceinline__ int predict_level(const plvi_frustum_params& p, float ratio) {
    if (__builtin_isinf(ratio)) return 0;  // ceil(inf) -> cvttss2si INT_MIN -> nScale < 0 -> 0
    int l = 0;
    for (int n = 1; n < p.nlevels; ++n) l += ratio >= p.level_ratio[n];
    return l;
}

struct SideOut {
    float u, v, view_cos, depth;
    int level;
    bool in_view;
};

// isInFrustumChecks(pMP, limit, bRight) (Frame.cc:1751-1824) for camera c;
// with `mono` the Nleft == -1 body (:760-835), which differs only in what it
// stores and when (handled by the caller through u / v / reached_uv).
__device__ __forceinline__ SideOut frustum_side(const plvi_frustum_params& p, const plvi_frustum_camera& c, float px,
                                                float py, float pz, const float* nrm, float dmin, float dmax,
                                                bool fma_form, bool& reached_uv, float& invz) {
    SideOut o{};
    o.in_view = false;
    reached_uv = false;
    const float x = pose_row(c.R + 0, px, py, pz, c.t[0], fma_form);
    const float y = pose_row(c.R + 3, px, py, pz, c.t[1], fma_form);
    const float z = pose_row(c.R + 6, px, py, pz, c.t[2], fma_form);
    const double pc_dist = cv_norm3(x, y, z);
    invz = 1.0f / z;
    if (z < 0.0f) return o;
    float u, v;
    cam_project(c, x, y, z, u, v);
    if (u < p.min_x || u > p.max_x) return o;
    if (v < p.min_y || v > p.max_y) return o;
    o.u = u;
    o.v = v;
    reached_uv = true;
    const float max_d = 1.2f * dmax, min_d = 0.8f * dmin;
    const float ox = px - c.O[0], oy = py - c.O[1], oz = pz - c.O[2];
    const float dist = (float)cv_norm3(ox, oy, oz);
    if (dist < min_d || dist > max_d) return o;
    const float view_cos = (float)(cv_dot3(ox, oy, oz, nrm[0], nrm[1], nrm[2]) / (double)dist);
    if (view_cos < p.view_cos_limit) return o;
    o.level = predict_level(p, dmax / dist);
    o.view_cos = view_cos;
    o.depth = (float)pc_dist;
    o.in_view = true;
    return o;
}

__global__ __launch_bounds__(256) void frustum_points_kernel(
    const plvi_frustum_params* __restrict__ params, const float* __restrict__ pos, const float* __restrict__ normal,
    const float* __restrict__ dist, const uint8_t* __restrict__ in_flags, const int* __restrict__ counts, int cap,
    uint8_t* __restrict__ flags, float* __restrict__ proj, int* __restrict__ level, float* __restrict__ proj_r,
    int* __restrict__ level_r, float* __restrict__ depth, int* __restrict__ nvisible) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = counts[f];
    if (i >= n || i >= cap) return;
    const plvi_frustum_params& p = params[f];
    const size_t k = (size_t)f * cap + i;
    const uint8_t fin = in_flags[k];
    uint8_t fo = fin & PLVI_FRUSTUM_OBS;
    if (!(fin & 1)) {
        flags[k] = fo;
        return;
    }
    const float px = pos[3 * k], py = pos[3 * k + 1], pz = pos[3 * k + 2];
    const float nrm[3] = {normal[3 * k], normal[3 * k + 1], normal[3 * k + 2]};
    const float dmin = dist[2 * k], dmax = dist[2 * k + 1];
    const bool fma_form = (p.compat & PLVI_COMPAT_GEMM_FMA) != 0;
    float* P = proj + 4 * k;
    bool visible, track, search_l, search_r = false;
    float invz;
    bool reached;
    if (!p.two_camera) {
        // Frame.cc:760-835
        const SideOut o = frustum_side(p, p.cam[0], px, py, pz, nrm, dmin, dmax, fma_form, reached, invz);
        P[0] = reached ? o.u : -1.0f;
        P[1] = reached ? o.v : -1.0f;
        if (o.in_view) {
            P[2] = rfmaf(-p.mbf, invz, o.u);  // uv.x - mbf*invz, fused in Frame.cc.o
            P[3] = o.view_cos;
            depth[k] = o.depth;
            level[k] = o.level;
        }
        visible = track = o.in_view;
        search_l = o.in_view && !(p.far_points && depth[k] > p.far_th);
    } else {
        // Frame.cc:836-846: both cameras, levels reset to -1 first
        const SideOut l = frustum_side(p, p.cam[0], px, py, pz, nrm, dmin, dmax, fma_form, reached, invz);
        const SideOut r = frustum_side(p, p.cam[1], px, py, pz, nrm, dmin, dmax, fma_form, reached, invz);
        level[k] = l.in_view ? l.level : -1;
        if (level_r) level_r[k] = r.in_view ? r.level : -1;
        if (l.in_view) {
            P[0] = l.u;
            P[1] = l.v;
            P[3] = l.view_cos;
            depth[k] = l.depth;
        }
        if (r.in_view && proj_r) {
            float* Q = proj_r + 4 * k;
            Q[0] = r.u;
            Q[1] = r.v;
            Q[3] = r.view_cos;
        }
        visible = l.in_view || r.in_view;
        track = l.in_view;
        // SearchByProjection's far test reads mTrackDepth, stale when only
        // the right camera sees the point (ORBmatcher.cc:56)
        const bool near = !(p.far_points && depth[k] > p.far_th);
        search_l = l.in_view && near;
        search_r = r.in_view && near;
    }
    fo |= (search_l ? PLVI_FRUSTUM_SEARCH : 0) | (search_r ? PLVI_FRUSTUM_SEARCH_R : 0) |
          (visible ? PLVI_FRUSTUM_VISIBLE : 0) | (track ? PLVI_FRUSTUM_TRACK : 0);
    flags[k] = fo;
    if (nvisible && visible) atomicAdd(&nvisible[f], 1);
}

// isInFrustum_l for line i of frame p; proj written as the reference writes
// mTrackProjs / mTrackProje (each once its endpoint passed).
__device__ bool frustum_line(const plvi_frustum_params& p, const double* sep, const float* nrm, float dmin, float dmax,
                             float* P, double* angle) {
    const plvi_frustum_camera& c = p.cam[0];
    const bool fma_form = (p.compat & PLVI_COMPAT_GEMM_FMA) != 0;
    float uv[4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        // Converter::toCvMat(Vector3d): element-wise float conversion
        const float X = (float)sep[3 * e], Y = (float)sep[3 * e + 1], Z = (float)sep[3 * e + 2];
        const float x = pose_row(c.R + 0, X, Y, Z, c.t[0], fma_form);
        const float y = pose_row(c.R + 3, X, Y, Z, c.t[1], fma_form);
        const float z = pose_row(c.R + 6, X, Y, Z, c.t[2], fma_form);
        if (z < 0.0f) return false;
        const float invz = 1.0f / z;
        const float u = rfmaf(c.fx * x, invz, c.cx);  // fx*PcX*invz + cx, fused in Frame.cc.o
        const float v = rfmaf(c.fy * y, invz, c.cy);
        if (u < p.min_x || u > p.max_x) return false;
        if (v < p.min_y || v > p.max_y) return false;
        P[2 * e] = u;
        P[2 * e + 1] = v;
        uv[2 * e] = u;
        uv[2 * e + 1] = v;
    }
    // MidPoint = (sp + ep) / 2 in double, then toCvMat
    const float mx = (float)((sep[0] + sep[3]) / 2), my = (float)((sep[1] + sep[4]) / 2),
                mz = (float)((sep[2] + sep[5]) / 2);
    const float max_d = 1.2f * dmax, min_d = 0.8f * dmin;
    const float ox = mx - c.O[0], oy = my - c.O[1], oz = mz - c.O[2];
    const float dist = (float)cv_norm3(ox, oy, oz);
    if (dist < min_d || dist > max_d) return false;
    const float view_cos = (float)(cv_dot3(ox, oy, oz, nrm[0], nrm[1], nrm[2]) / (double)dist);
    if (view_cos < p.view_cos_limit) return false;
    // atan2(float, float) = atan2f, stored in the double mnTrackangle
    *angle = (double)plvi_atan2f(uv[3] - uv[1], uv[2] - uv[0]);
    return true;
}

__global__ __launch_bounds__(256) void frustum_lines_kernel(
    const plvi_frustum_params* __restrict__ params, const double* __restrict__ sep, const float* __restrict__ normal,
    const float* __restrict__ dist, const uint8_t* __restrict__ in_flags, const uint8_t* __restrict__ desc,
    const int* __restrict__ counts, int cap, uint8_t* __restrict__ inview, float* __restrict__ proj,
    double* __restrict__ angle, int* __restrict__ compact, uint8_t* __restrict__ compact_desc,
    int* __restrict__ ncompact) {
    __shared__ int s_wave[4];
    __shared__ int s_base;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const plvi_frustum_params& p = params[f];
    const int n = min(counts[f], cap);
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += 256) {
        const int i = i0 + tid;
        bool in = false;
        if (i < n) {
            const size_t k = (size_t)f * cap + i;
            if (in_flags[k] & 1)
                in = frustum_line(p, sep + 6 * k, normal + 3 * k, dist[2 * k], dist[2 * k + 1], proj + 4 * k,
                                  angle + k);
            inview[k] = in;
        }
        const unsigned long long m = __ballot(in);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) s_wave[wv] = __popcll(m);
        __syncthreads();
        int off = s_base;
        for (int w = 0; w < wv; ++w) off += s_wave[w];
        if (in) {
            const int j = off + before;
            const size_t o = (size_t)f * cap + j;
            compact[o] = i;
            if (desc && compact_desc) {
                const uint4* s = reinterpret_cast<const uint4*>(desc + 32 * ((size_t)f * cap + i));
                uint4* d = reinterpret_cast<uint4*>(compact_desc + 32 * o);
                d[0] = s[0];
                d[1] = s[1];
            }
        }
        __syncthreads();
        if (tid == 0) s_base += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        __syncthreads();
    }
    if (tid == 0) ncompact[f] = s_base;
}

// Tracking.cc:5247-5292 for frame f: one thread per in-frustum line i1.
// matches_12 is one-to-one after the cross check (LineMatcher::match), so the
// loop's order does not matter: each i2 is visited at most once.
__global__ __launch_bounds__(256) void local_lines_filter_kernel(
    const plvi_frustum_params* __restrict__ params, int* __restrict__ matches, const int* __restrict__ ncompact,
    const int* __restrict__ compact, int cap, const float* __restrict__ proj, const double* __restrict__ angle,
    const plvi_keyline* __restrict__ kl, const int* __restrict__ nkl, int kl_cap, const uint8_t* __restrict__ blocked,
    int* __restrict__ assign, int* __restrict__ nassigned) {
    const int f = blockIdx.y;
    const int i1 = blockIdx.x * 256 + threadIdx.x;
    const int nc = min(ncompact[f], cap);
    if (i1 >= nc) return;
    const plvi_frustum_params& p = params[f];
    int* M = matches + (size_t)f * cap;
    const int i2 = M[i1];
    if (i2 < 0 || i2 >= min(nkl[f], kl_cap)) return;
    const size_t k2 = (size_t)f * kl_cap + i2;
    if (blocked && blocked[k2]) return;
    const int il = compact[(size_t)f * cap + i1];
    const size_t kl1 = (size_t)f * cap + il;
    const plvi_keyline& K = kl[k2];
    const double kPi = 3.14159265358979323846;
    const double delta_angle = kPi / 10.0;
    const double delta_w = (double)(p.max_x - p.min_x) * 0.1;
    const double delta_h = (double)(p.max_y - p.min_y) * 0.1;
    const double theta1 = (double)plvi_atan2f(K.endPointY - K.startPointY, K.endPointX - K.startPointX);
    double theta = theta1 - angle[kl1];
    if (theta < -kPi) theta += 2 * kPi;
    else if (theta > kPi) theta -= 2 * kPi;
    if (__builtin_fabs(theta) > delta_angle) {
        M[i1] = -1;
        return;
    }
    const float* P = proj + 4 * kl1;
    if ((double)__builtin_fabsf(K.startPointX - P[0]) > delta_w || (double)__builtin_fabsf(K.endPointX - P[2]) > delta_w ||
        (double)__builtin_fabsf(K.startPointY - P[1]) > delta_h || (double)__builtin_fabsf(K.endPointY - P[3]) > delta_h) {
        M[i1] = -1;
        return;
    }
    assign[k2] = il;
    atomicAdd(&nassigned[f], 1);
}

// PredictScale exactly as MapPoint.cc.o: logf, vdivss, vroundss (ceil),
// vcvttss2si (INT_MIN out of range / NaN), clamp.
int predict_level_host(float ratio, float lsf, int nlevels) {
    const float q = std::ceil(logf(ratio) / lsf);
    int s;
    if (!(q >= -2147483648.0f && q < 2147483648.0f)) s = INT32_MIN;
    else s = (int)q;
    if (s < 0) s = 0;
    else if (s >= nlevels) s = nlevels - 1;
    return s;
}

}  // namespace

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_frustum_params_init(plvi_frustum_params* p) {
    if (!p || p->nlevels < 1 || p->nlevels > 16) return PLVI_E_BADARG;
    const float lsf = p->log_scale_factor;
    if (!(lsf >= 0.0f)) return PLVI_E_BADARG;
    p->level_ratio[0] = -INFINITY;
    for (int n = 1; n < 16; ++n) {
        p->level_ratio[n] = INFINITY;
        if (n >= p->nlevels) continue;
        // least positive finite float with level >= n (level is monotone in
        // the ratio: tests/test_frustum.py checks every float around each
        // threshold against the direct formula)
        uint32_t lo = f2u(1.0f), hi = f2u(3.4028235e38f);
        if (predict_level_host(u2f(hi), lsf, p->nlevels) < n) continue;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (predict_level_host(u2f(mid), lsf, p->nlevels) >= n) hi = mid;
            else lo = mid + 1;
        }
        p->level_ratio[n] = u2f(lo);
    }
    return PLVI_OK;
}

extern "C" int plvi_frustum_points_batch(int n_frames, const plvi_frustum_params* d_params, const float* d_pos,
                                         const float* d_normal, const float* d_dist, const uint8_t* d_in_flags,
                                         const int* d_n, int cap, uint8_t* d_flags, float* d_proj, int* d_level,
                                         float* d_proj_r, int* d_level_r, float* d_depth, int* d_nvisible,
                                         void* stream) {
    if (n_frames < 0 || cap < 1 || n_frames > 65535) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    if (!d_params || !d_pos || !d_normal || !d_dist || !d_in_flags || !d_n || !d_flags || !d_proj || !d_level ||
        !d_depth)
        return PLVI_E_BADARG;
    hipStream_t st = (hipStream_t)stream;
    if (d_nvisible) PLVI_CHECK(hipMemsetAsync(d_nvisible, 0, sizeof(int) * n_frames, st));
    hipLaunchKernelGGL(frustum_points_kernel, dim3((cap + 255) / 256, n_frames), dim3(256), 0, st, d_params, d_pos,
                       d_normal, d_dist, d_in_flags, d_n, cap, d_flags, d_proj, d_level, d_proj_r, d_level_r, d_depth,
                       d_nvisible);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

namespace {
// Device scratch of the synchronous one-frame entry points.
struct Slots {
    std::vector<size_t> off;
    size_t tot = 0;
    size_t put(size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    }
};
}  // namespace

extern "C" int plvi_frustum_points(const plvi_frustum_params* p, const float* pos, const float* normal,
                                   const float* dist, const uint8_t* in_flags, int n, uint8_t* flags, float* proj,
                                   int* level, float* proj_r, int* level_r, float* depth) {
    if (!p || n < 0) return PLVI_E_BADARG;
    if (n == 0) return 0;
    if (!pos || !normal || !dist || !in_flags || !flags || !proj || !level || !depth) return PLVI_E_BADARG;
    if (p->two_camera && (!proj_r || !level_r)) return PLVI_E_BADARG;
    Slots s;
    const size_t oPar = s.put(sizeof(plvi_frustum_params)), oPos = s.put(12 * (size_t)n), oNr = s.put(12 * (size_t)n);
    const size_t oD = s.put(8 * (size_t)n), oIF = s.put(n), oF = s.put(n), oP = s.put(16 * (size_t)n);
    const size_t oL = s.put(4 * (size_t)n), oPR = s.put(16 * (size_t)n), oLR = s.put(4 * (size_t)n);
    const size_t oDe = s.put(4 * (size_t)n), oN = s.put(8);
    DevBuf d;
    if (d.alloc(s.tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        PLVI_CHECK(hipMemcpy(B + s.off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oPar, p, sizeof *p) | up(oPos, pos, 12 * (size_t)n) | up(oNr, normal, 12 * (size_t)n) |
             up(oD, dist, 8 * (size_t)n) | up(oIF, in_flags, n) | up(oP, proj, 16 * (size_t)n) |
             up(oL, level, 4 * (size_t)n) | up(oDe, depth, 4 * (size_t)n);
    if (p->two_camera) rc |= up(oPR, proj_r, 16 * (size_t)n) | up(oLR, level_r, 4 * (size_t)n);
    rc |= up(oN, &n, 4);
    if (rc) return PLVI_E_HIP;
    int* dN = reinterpret_cast<int*>(B + s.off[oN]);
    rc = plvi_frustum_points_batch(1, reinterpret_cast<const plvi_frustum_params*>(B + s.off[oPar]),
                                   reinterpret_cast<const float*>(B + s.off[oPos]),
                                   reinterpret_cast<const float*>(B + s.off[oNr]),
                                   reinterpret_cast<const float*>(B + s.off[oD]), B + s.off[oIF], dN, n, B + s.off[oF],
                                   reinterpret_cast<float*>(B + s.off[oP]), reinterpret_cast<int*>(B + s.off[oL]),
                                   p->two_camera ? reinterpret_cast<float*>(B + s.off[oPR]) : nullptr,
                                   p->two_camera ? reinterpret_cast<int*>(B + s.off[oLR]) : nullptr,
                                   reinterpret_cast<float*>(B + s.off[oDe]), dN + 1, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nvis = 0;
    PLVI_CHECK(hipMemcpy(flags, B + s.off[oF], n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(proj, B + s.off[oP], 16 * (size_t)n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(level, B + s.off[oL], 4 * (size_t)n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(depth, B + s.off[oDe], 4 * (size_t)n, hipMemcpyDeviceToHost));
    if (p->two_camera) {
        PLVI_CHECK(hipMemcpy(proj_r, B + s.off[oPR], 16 * (size_t)n, hipMemcpyDeviceToHost));
        PLVI_CHECK(hipMemcpy(level_r, B + s.off[oLR], 4 * (size_t)n, hipMemcpyDeviceToHost));
    }
    PLVI_CHECK(hipMemcpy(&nvis, dN + 1, 4, hipMemcpyDeviceToHost));
    return nvis;
}

extern "C" int plvi_frustum_lines_batch(int n_frames, const plvi_frustum_params* d_params, const double* d_sep,
                                        const float* d_normal, const float* d_dist, const uint8_t* d_in_flags,
                                        const uint8_t* d_desc, const int* d_n, int cap, uint8_t* d_inview,
                                        float* d_proj, double* d_angle, int* d_compact, uint8_t* d_compact_desc,
                                        int* d_ncompact, void* stream) {
    if (n_frames < 0 || cap < 1) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    if (!d_params || !d_sep || !d_normal || !d_dist || !d_in_flags || !d_n || !d_inview || !d_proj || !d_angle ||
        !d_compact || !d_ncompact)
        return PLVI_E_BADARG;
    hipLaunchKernelGGL(frustum_lines_kernel, dim3(n_frames), dim3(256), 0, (hipStream_t)stream, d_params, d_sep,
                       d_normal, d_dist, d_in_flags, d_desc, d_n, cap, d_inview, d_proj, d_angle, d_compact,
                       d_compact_desc, d_ncompact);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_frustum_lines(const plvi_frustum_params* p, const double* sep, const float* normal,
                                  const float* dist, const uint8_t* in_flags, const uint8_t* desc, int n,
                                  uint8_t* inview, float* proj, double* angle, int* compact, uint8_t* compact_desc) {
    if (!p || n < 0) return PLVI_E_BADARG;
    if (n == 0) return 0;
    if (!sep || !normal || !dist || !in_flags || !inview || !proj || !angle || !compact) return PLVI_E_BADARG;
    Slots s;
    const size_t oPar = s.put(sizeof(plvi_frustum_params)), oS = s.put(48 * (size_t)n), oNr = s.put(12 * (size_t)n);
    const size_t oD = s.put(8 * (size_t)n), oIF = s.put(n), oDs = s.put(32 * (size_t)n), oIV = s.put(n);
    const size_t oP = s.put(16 * (size_t)n), oA = s.put(8 * (size_t)n), oC = s.put(4 * (size_t)n);
    const size_t oCD = s.put(32 * (size_t)n), oN = s.put(8);
    DevBuf d;
    if (d.alloc(s.tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        PLVI_CHECK(hipMemcpy(B + s.off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oPar, p, sizeof *p) | up(oS, sep, 48 * (size_t)n) | up(oNr, normal, 12 * (size_t)n) |
             up(oD, dist, 8 * (size_t)n) | up(oIF, in_flags, n) | up(oP, proj, 16 * (size_t)n) |
             up(oA, angle, 8 * (size_t)n) | up(oN, &n, 4);
    if (desc) rc |= up(oDs, desc, 32 * (size_t)n);
    if (rc) return PLVI_E_HIP;
    int* dN = reinterpret_cast<int*>(B + s.off[oN]);
    rc = plvi_frustum_lines_batch(1, reinterpret_cast<const plvi_frustum_params*>(B + s.off[oPar]),
                                  reinterpret_cast<const double*>(B + s.off[oS]),
                                  reinterpret_cast<const float*>(B + s.off[oNr]),
                                  reinterpret_cast<const float*>(B + s.off[oD]), B + s.off[oIF],
                                  desc ? B + s.off[oDs] : nullptr, dN, n, B + s.off[oIV],
                                  reinterpret_cast<float*>(B + s.off[oP]), reinterpret_cast<double*>(B + s.off[oA]),
                                  reinterpret_cast<int*>(B + s.off[oC]), desc ? B + s.off[oCD] : nullptr, dN + 1,
                                  nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nc = 0;
    PLVI_CHECK(hipMemcpy(&nc, dN + 1, 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(inview, B + s.off[oIV], n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(proj, B + s.off[oP], 16 * (size_t)n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(angle, B + s.off[oA], 8 * (size_t)n, hipMemcpyDeviceToHost));
    if (nc > 0) {
        PLVI_CHECK(hipMemcpy(compact, B + s.off[oC], 4 * (size_t)nc, hipMemcpyDeviceToHost));
        if (desc && compact_desc)
            PLVI_CHECK(hipMemcpy(compact_desc, B + s.off[oCD], 32 * (size_t)nc, hipMemcpyDeviceToHost));
    }
    return nc;
}

extern "C" int plvi_local_lines_filter_batch(int n_frames, const plvi_frustum_params* d_params, int* d_matches_12,
                                             const int* d_ncompact, const int* d_compact, int cap, const float* d_proj,
                                             const double* d_angle, const plvi_keyline* d_kl, const int* d_nkl,
                                             int kl_cap, const uint8_t* d_blocked, int* d_assign, int* d_nassigned,
                                             void* stream) {
    if (n_frames < 0 || cap < 1 || kl_cap < 1 || n_frames > 65535) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    if (!d_params || !d_matches_12 || !d_ncompact || !d_compact || !d_proj || !d_angle || !d_kl || !d_nkl ||
        !d_assign || !d_nassigned)
        return PLVI_E_BADARG;
    hipStream_t st = (hipStream_t)stream;
    PLVI_CHECK(hipMemsetAsync(d_assign, 0xFF, sizeof(int) * (size_t)n_frames * kl_cap, st));
    PLVI_CHECK(hipMemsetAsync(d_nassigned, 0, sizeof(int) * n_frames, st));
    hipLaunchKernelGGL(local_lines_filter_kernel, dim3((cap + 255) / 256, n_frames), dim3(256), 0, st, d_params,
                       d_matches_12, d_ncompact, d_compact, cap, d_proj, d_angle, d_kl, d_nkl, kl_cap, d_blocked,
                       d_assign, d_nassigned);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}
