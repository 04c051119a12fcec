// oracle/frustum_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the local-map visibility test and the local line filter
// of Tracking::SearchLocalPoints / SearchLocalPointsAndLines
// (src/Tracking.cc:5074-5092, :5166-5184, :5214-5292):
//   Frame::isInFrustum(pMP, viewingCosLimit)   src/Frame.cc:758-835 (Nleft == -1)
//                                              :836-846 + isInFrustumChecks :1751-1824 (Nleft != -1)
//   Frame::isInFrustum_l(pML, viewingCosLimit) src/Frame.cc:849-933
//   MapPoint::PredictScale(dist, Frame*)       src/MapPoint.cc:531-546 (glibc logf, ceil, cvttss2si)
//   Get{Min,Max}DistanceInvariance             src/MapPoint.cc:502-512, src/MapLine.cc:384-394
//   Converter::toCvMat(Vector3d)               src/Converter.cc:91-98
//   Pinhole / KannalaBrandt8 project           src/CameraModels/Pinhole.cpp:30-39,
//                                              KannalaBrandt8.cpp:28-50
// Pinned by the shipped objects (tests/test_ref_objects.py): the fused
// multiply-adds of Frame.cc.o (mTrackProjXR, the four isInFrustum_l
// endpoint coordinates) and KannalaBrandt8.cpp.o, PredictScale's instruction
// sequence, the float / double conversions around cv::norm and Mat::dot.
// Parity unpinned: OpenCV's own arithmetic inside cv::gemm (3x3 * 3x1 + 3x1
// small-matrix path: float products and sums, then double alpha / beta;
// PLVI_COMPAT_GEMM_FMA = its AVX2-dispatched contraction), cv::norm (exact
// float squares summed in double) and Mat::dot (exact products in double) --
// the IPP paths of an IPP-enabled OpenCV build could order those sums
// differently.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/plvi_frontend.h"
#include "ref_fma.h"

namespace {

struct V3 {
    float x, y, z;
};

// mR*P + mt through cv::gemm's small-matrix path
V3 gemm_pose(const plvi_frustum_camera& c, const V3& P, bool fma_form) {
    auto row = [&](const float* a, float t) {
        float s;
        if (fma_form) s = ref_fmaf(a[2], P.z, ref_fmaf(a[0], P.x, a[1] * P.y));
        else s = a[0] * P.x + a[1] * P.y + a[2] * P.z;
        const double t0 = s;
        return (float)(t0 * 1.0 + (double)t * 1.0);  // (float)(t0*alpha + c[0]*beta)
    };
    return {row(c.R, c.t[0]), row(c.R + 3, c.t[1]), row(c.R + 6, c.t[2])};
}

double cv_norm(const V3& v) {  // normL2Sqr<float, double> + std::sqrt
    double s = 0;
    const float a[3] = {v.x, v.y, v.z};
    for (int i = 0; i < 3; i++) {
        double t = a[i];
        s += t * t;
    }
    return std::sqrt(s);
}

double cv_dot(const V3& a, const V3& b) {  // dotProd_<float>
    double r = 0;
    r += (double)a.x * b.x;
    r += (double)a.y * b.y;
    r += (double)a.z * b.z;
    return r;
}

void project(const plvi_frustum_camera& c, const V3& p, float& u, float& v) {
    if (!c.model) {
        u = c.fx * p.x / p.z + c.cx;
        v = c.fy * p.y / p.z + c.cy;
        return;
    }
    const float x2_plus_y2 = ref_fmaf(p.x, p.x, p.y * p.y);
    const float theta = atan2f(sqrtf(x2_plus_y2), p.z);
    const float psi = atan2f(p.y, p.x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r =
        ref_fmaf(c.kb[3], theta9, ref_fmaf(c.kb[2], theta7, ref_fmaf(c.kb[1], theta5, ref_fmaf(c.kb[0], theta3, theta))));
    u = ref_fmaf(c.fx * r, std::cos(psi), c.cx);
    v = ref_fmaf(c.fy * r, std::sin(psi), c.cy);
}

// MapPoint::PredictScale (MapPoint.cc:531-546) as MapPoint.cc.o computes it:
// logf, vdivss, vroundss $0xa (ceil), vcvttss2si (INT_MIN when out of range).
int predict_scale(float max_distance, float current_dist, float log_scale_factor, int nlevels) {
    const float ratio = max_distance / current_dist;
    const float q = std::ceil(logf(ratio) / log_scale_factor);
    int nScale = (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT32_MIN;
    if (nScale < 0) nScale = 0;
    else if (nScale >= nlevels) nScale = nlevels - 1;
    return nScale;
}

struct MP {
    // MapPoint state read / written by isInFrustum
    bool mbTrackInView, mbTrackInViewR;
    float mTrackProjX, mTrackProjY, mTrackProjXR, mTrackProjYR, mTrackViewCos, mTrackViewCosR, mTrackDepth;
    int mnTrackScaleLevel, mnTrackScaleLevelR;
};

// Frame::isInFrustumChecks (Frame.cc:1751-1824)
bool frustum_checks(const plvi_frustum_params& F, const V3& P, const V3& Pn, float mfMin, float mfMax, MP& m,
                    bool bRight) {
    const plvi_frustum_camera& c = F.cam[bRight ? 1 : 0];
    const bool fma_form = (F.compat & PLVI_COMPAT_GEMM_FMA) != 0;
    const V3 Pc = gemm_pose(c, P, fma_form);
    const float Pc_dist = (float)cv_norm(Pc);
    const float PcZ = Pc.z;
    if (PcZ < 0.0f) return false;
    float ux, uy;
    project(c, Pc, ux, uy);
    if (ux < F.min_x || ux > F.max_x) return false;
    if (uy < F.min_y || uy > F.max_y) return false;
    const float maxDistance = 1.2f * mfMax;
    const float minDistance = 0.8f * mfMin;
    const V3 PO{P.x - c.O[0], P.y - c.O[1], P.z - c.O[2]};
    const float dist = (float)cv_norm(PO);
    if (dist < minDistance || dist > maxDistance) return false;
    const float viewCos = (float)(cv_dot(PO, Pn) / dist);
    if (viewCos < F.view_cos_limit) return false;
    const int nPredictedLevel = predict_scale(mfMax, dist, F.log_scale_factor, F.nlevels);
    if (bRight) {
        m.mTrackProjXR = ux;
        m.mTrackProjYR = uy;
        m.mnTrackScaleLevelR = nPredictedLevel;
        m.mTrackViewCosR = viewCos;
    } else {
        m.mTrackProjX = ux;
        m.mTrackProjY = uy;
        m.mnTrackScaleLevel = nPredictedLevel;
        m.mTrackViewCos = viewCos;
        m.mTrackDepth = Pc_dist;
    }
    return true;
}

// Frame::isInFrustum (Frame.cc:758-847)
bool is_in_frustum(const plvi_frustum_params& F, const V3& P, const V3& Pn, float mfMin, float mfMax, MP& m) {
    if (F.two_camera) {
        m.mbTrackInView = false;
        m.mbTrackInViewR = false;
        m.mnTrackScaleLevel = -1;
        m.mnTrackScaleLevelR = -1;
        m.mbTrackInView = frustum_checks(F, P, Pn, mfMin, mfMax, m, false);
        m.mbTrackInViewR = frustum_checks(F, P, Pn, mfMin, mfMax, m, true);
        return m.mbTrackInView || m.mbTrackInViewR;
    }
    const plvi_frustum_camera& c = F.cam[0];
    m.mbTrackInView = false;
    m.mTrackProjX = -1;
    m.mTrackProjY = -1;
    const V3 Pc = gemm_pose(c, P, (F.compat & PLVI_COMPAT_GEMM_FMA) != 0);
    const float Pc_dist = (float)cv_norm(Pc);
    const float PcZ = Pc.z;
    const float invz = 1.0f / PcZ;
    if (PcZ < 0.0f) return false;
    float ux, uy;
    project(c, Pc, ux, uy);
    if (ux < F.min_x || ux > F.max_x) return false;
    if (uy < F.min_y || uy > F.max_y) return false;
    m.mTrackProjX = ux;
    m.mTrackProjY = uy;
    const float maxDistance = 1.2f * mfMax;
    const float minDistance = 0.8f * mfMin;
    const V3 PO{P.x - c.O[0], P.y - c.O[1], P.z - c.O[2]};
    const float dist = (float)cv_norm(PO);
    if (dist < minDistance || dist > maxDistance) return false;
    const float viewCos = (float)(cv_dot(PO, Pn) / dist);
    if (viewCos < F.view_cos_limit) return false;
    const int nPredictedLevel = predict_scale(mfMax, dist, F.log_scale_factor, F.nlevels);
    m.mbTrackInView = true;
    m.mTrackProjX = ux;
    m.mTrackProjXR = ref_fmaf(-F.mbf, invz, ux);  // uv.x - mbf*invz (vfnmadd132ss in Frame.cc.o)
    m.mTrackDepth = Pc_dist;
    m.mTrackProjY = uy;
    m.mnTrackScaleLevel = nPredictedLevel;
    m.mTrackViewCos = viewCos;
    return true;
}

}  // namespace

extern "C" int oracle_predict_scale(float max_distance, float current_dist, float log_scale_factor, int nlevels) {
    return predict_scale(max_distance, current_dist, log_scale_factor, nlevels);
}

// Every float ratio r in [lo, hi] (positive): PredictScale(r) (as max / 1)
// against the table rule #{n : r >= thr[n]}; returns the number of
// mismatches (the first one's bits in *first).
extern "C" long long oracle_level_table_check(const float* thr, float lsf, int nlevels, float lo, float hi,
                                              uint32_t* first) {
    uint32_t a, b;
    std::memcpy(&a, &lo, 4);
    std::memcpy(&b, &hi, 4);
    long long bad = 0;
    for (uint32_t u = a; u <= b; ++u) {
        float r;
        std::memcpy(&r, &u, 4);
        const float q = std::ceil(logf(r) / lsf);
        int s = (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT32_MIN;
        if (s < 0) s = 0;
        else if (s >= nlevels) s = nlevels - 1;
        int t = 0;
        if (!std::isinf(r))
            for (int n = 1; n < nlevels; ++n) t += r >= thr[n];
        if (s != t) {
            if (!bad && first) *first = u;
            ++bad;
        }
        if (u == 0xFFFFFFFFu) break;
    }
    return bad;
}

// The local MapPoints of one frame through Tracking.cc:5074-5092 and the
// entry tests of ORBmatcher::SearchByProjection (ORBmatcher.cc:50-60).
// Buffers as plvi_frustum_points (proj / level / proj_r / level_r / depth
// in/out: the MapPoint fields before the call).  Returns nToMatch.
extern "C" int oracle_frustum_points(const plvi_frustum_params* F, const float* pos, const float* normal,
                                     const float* dist, const uint8_t* in_flags, int n, uint8_t* flags, float* proj,
                                     int* level, float* proj_r, int* level_r, float* depth) {
    int nToMatch = 0;
    for (int i = 0; i < n; ++i) {
        uint8_t fo = in_flags[i] & PLVI_FRUSTUM_OBS;
        if (!(in_flags[i] & 1)) {  // mnLastFrameSeen == mnId or isBad(): not searched
            flags[i] = fo;
            continue;
        }
        MP m{};
        m.mTrackProjX = proj[4 * i];
        m.mTrackProjY = proj[4 * i + 1];
        m.mTrackProjXR = proj[4 * i + 2];
        m.mTrackViewCos = proj[4 * i + 3];
        m.mnTrackScaleLevel = level[i];
        m.mTrackDepth = depth[i];
        if (F->two_camera) {
            m.mTrackProjXR = proj_r[4 * i];
            m.mTrackProjYR = proj_r[4 * i + 1];
            m.mTrackViewCosR = proj_r[4 * i + 3];
            m.mnTrackScaleLevelR = level_r[i];
        }
        const V3 P{pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]};
        const V3 Pn{normal[3 * i], normal[3 * i + 1], normal[3 * i + 2]};
        const bool vis = is_in_frustum(*F, P, Pn, dist[2 * i], dist[2 * i + 1], m);
        if (vis) {
            nToMatch++;
            fo |= PLVI_FRUSTUM_VISIBLE;
        }
        if (m.mbTrackInView) fo |= PLVI_FRUSTUM_TRACK;
        // SearchByProjection: skip !mbTrackInView && !mbTrackInViewR, far (mTrackDepth)
        const bool far = F->far_points && m.mTrackDepth > F->far_th;
        if (m.mbTrackInView && !far) fo |= PLVI_FRUSTUM_SEARCH;
        if (F->two_camera && m.mbTrackInViewR && !far) fo |= PLVI_FRUSTUM_SEARCH_R;
        flags[i] = fo;
        proj[4 * i] = m.mTrackProjX;
        proj[4 * i + 1] = m.mTrackProjY;
        if (!F->two_camera) proj[4 * i + 2] = m.mTrackProjXR;
        proj[4 * i + 3] = m.mTrackViewCos;
        level[i] = m.mnTrackScaleLevel;
        depth[i] = m.mTrackDepth;
        if (F->two_camera) {
            proj_r[4 * i] = m.mTrackProjXR;
            proj_r[4 * i + 1] = m.mTrackProjYR;
            proj_r[4 * i + 3] = m.mTrackViewCosR;
            level_r[i] = m.mnTrackScaleLevelR;
        }
    }
    return nToMatch;
}

// Frame::isInFrustum_l (Frame.cc:849-933) over one frame's local MapLines
// (Tracking.cc:5219-5234).  Buffers as plvi_frustum_lines (proj / angle in/out).
// Returns nToMatch = the length of compact (mvpLocalMapLines_InFrustum).
extern "C" int oracle_frustum_lines(const plvi_frustum_params* F, const double* sep, const float* normal,
                                    const float* dist, const uint8_t* in_flags, int n, uint8_t* inview, float* proj,
                                    double* angle, int* compact) {
    const plvi_frustum_camera& c = F->cam[0];
    const bool fma_form = (F->compat & PLVI_COMPAT_GEMM_FMA) != 0;
    const float fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    int nToMatch = 0;
    for (int i = 0; i < n; ++i) {
        inview[i] = 0;
        if (!(in_flags[i] & 1)) continue;
        bool ok = true;
        const double* s = sep + 6 * i;
        float* pr = proj + 4 * i;
        for (int e = 0; e < 2 && ok; ++e) {
            const V3 p{(float)s[3 * e], (float)s[3 * e + 1], (float)s[3 * e + 2]};  // toCvMat
            const V3 Pc = gemm_pose(c, p, fma_form);
            const float PcX = Pc.x, PcY = Pc.y, PcZ = Pc.z;
            if (PcZ < 0.0f) {
                ok = false;
                break;
            }
            const float invz = 1.0f / PcZ;
            const float u = ref_fmaf(fx * PcX, invz, cx);  // fx*PcX*invz+cx (vfmadd213ss)
            const float v = ref_fmaf(fy * PcY, invz, cy);
            if (u < F->min_x || u > F->max_x || v < F->min_y || v > F->max_y) {
                ok = false;
                break;
            }
            pr[2 * e] = u;
            pr[2 * e + 1] = v;
        }
        if (!ok) continue;
        const double mid[3] = {(s[0] + s[3]) / 2, (s[1] + s[4]) / 2, (s[2] + s[5]) / 2};
        const V3 P{(float)mid[0], (float)mid[1], (float)mid[2]};
        const float maxDistance = 1.2f * dist[2 * i + 1];
        const float minDistance = 0.8f * dist[2 * i];
        const V3 PO{P.x - c.O[0], P.y - c.O[1], P.z - c.O[2]};
        const float d = (float)cv_norm(PO);
        if (d < minDistance || d > maxDistance) continue;
        const V3 Pn{normal[3 * i], normal[3 * i + 1], normal[3 * i + 2]};
        const float viewCos = (float)(cv_dot(PO, Pn) / d);
        if (viewCos < F->view_cos_limit) continue;
        inview[i] = 1;
        angle[i] = atan2f(pr[3] - pr[1], pr[2] - pr[0]);
        compact[nToMatch++] = i;
    }
    return nToMatch;
}

// Tracking.cc:5244-5292 for one frame: matches_12 over the in-frustum lines
// (in/out), keylines mvKeysUn_Line as (sx, sy, ex, ey) [nkl][4], blocked
// (nullable).  assign[nkl] = local MapLine index or -1.  Returns the count.
extern "C" int oracle_local_lines_filter(const plvi_frustum_params* F, int* matches_12, int nc, const int* compact,
                                         const float* proj, const double* angle, const float* kl, int nkl,
                                         const uint8_t* blocked, int* assign) {
    const double deltaAngle = M_PI / 10.0;
    const double deltaWidth = (F->max_x - F->min_x) * 0.1;
    const double deltaHeight = (F->max_y - F->min_y) * 0.1;
    for (int i = 0; i < nkl; ++i) assign[i] = -1;
    int na = 0;
    for (int i1 = 0; i1 < nc; ++i1) {
        const int i2 = matches_12[i1];
        if (i2 < 0) continue;
        if (blocked && blocked[i2]) continue;
        const int il = compact[i1];
        const float* k = kl + 4 * i2;
        double theta1 = atan2f(k[3] - k[1], k[2] - k[0]);
        double theta2 = angle[il];
        double theta = theta1 - theta2;
        if (theta < -M_PI) theta += 2 * M_PI;
        else if (theta > M_PI) theta -= 2 * M_PI;
        if (std::fabs(theta) > deltaAngle) {
            matches_12[i1] = -1;
            continue;
        }
        const float* pr = proj + 4 * il;
        if (std::fabs(k[0] - pr[0]) > deltaWidth || std::fabs(k[2] - pr[2]) > deltaWidth ||
            std::fabs(k[1] - pr[1]) > deltaHeight || std::fabs(k[3] - pr[3]) > deltaHeight) {
            matches_12[i1] = -1;
            continue;
        }
        assign[i2] = il;
        ++na;
    }
    return na;
}
