// proj.hip — the steady-state frame-to-frame ORB matcher on the device:
//   Frame::AssignFeaturesToGrid (src/Frame.cc:644-675) + PosInGrid (:1077-1087)
//   Frame::GetFeaturesInArea (src/Frame.cc:1006-1075)
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//     (src/ORBmatcher.cc:1962-2178, Nleft == -1 branch) + ComputeThreeMaxima
//   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, ...)
//     (src/ORBmatcher.cc:44-145, the local-map search)
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
//     (src/ORBmatcher.cc:2180-2300, the relocalization guided search)
// The pose product x3Dc = Rcw*x3Dw + tcw (cv::Mat float gemm) stays with the
// caller (drop-in shim); everything after it runs here.
//
// Grid kernel: one workgroup per frame; (cell << 13 | keypoint) keys sorted in
// LDS, so every cell lists its keypoints in index order as push_back does.
// CSR cell order = mGrid[ix][iy] with cell = ix * 48 + iy, so the cells of one
// grid column inside a search window are one contiguous index range.
//
// Matcher kernel: one workgroup per (CurrentFrame, LastFrame) pair.  The
// greedy assignment is sequential in LastFrame order only through one
// effect: a candidate that received a MapPoint with Observations() > 0 is
// skipped by later points (:2037-2039).  Phase 1 computes every point's best
// candidate in parallel (thread per point, the current frame's keypoints and
// grid in LDS) against the flags on entry; phase 2 walks the points in order
// and re-scans only a point whose best candidate was blocked meanwhile (the
// argmin over a subset that still contains it is unchanged otherwise);
// phase 3 is the rotation histogram filter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "plvi_common.h"
#include "plvi_math.h"

namespace plvi {

constexpr int kGridCols = 64, kGridRows = 48, kGridCells = kGridCols * kGridRows;  // include/Frame.h:47-48
constexpr int kProjThHigh = 100, kProjHisto = 30;
constexpr int kGridKeyBits = 13;  // keypoint index bits in the grid sort key (cap <= 8192)

__device__ __forceinline__ int round_half_away(float v) { return (int)roundf(v); }

__global__ __launch_bounds__(256) void assign_grid_kernel(const plvi_keypoint* __restrict__ kps,
                                                          const int* __restrict__ counts, int cap, int P,
                                                          plvi_grid_params gp, int* __restrict__ cell_off,
                                                          int* __restrict__ cell_idx) {
    extern __shared__ __align__(16) unsigned s_key[];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(counts[f], cap);
    const plvi_keypoint* K = kps + (size_t)f * cap;
    __shared__ int s_m;
    if (tid == 0) s_m = 0;
    __syncthreads();
    int cm = 0;
    for (int i = tid; i < P; i += 256) {
        unsigned key = 0xFFFFFFFFu;
        if (i < n) {
            // PosInGrid: std::round(float) of (pt - mnMin) * inv
            const int px = round_half_away((K[i].x - gp.min_x) * gp.inv_w);
            const int py = round_half_away((K[i].y - gp.min_y) * gp.inv_h);
            if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows)) {
                key = ((unsigned)(px * kGridRows + py) << kGridKeyBits) | (unsigned)i;
                ++cm;
            }
        }
        s_key[i] = key;
    }
    atomicAdd(&s_m, cm);
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < P / 2; t += 256) {
                const int i = (t / j) * 2 * j + (t % j), ixj = i + j;
                const bool asc = (i & k) == 0;
                const unsigned x = s_key[i], y = s_key[ixj];
                if ((x > y) == asc) {
                    s_key[i] = y;
                    s_key[ixj] = x;
                }
            }
            __syncthreads();
        }
    const int m = s_m;
    int* CO = cell_off + (size_t)f * (kGridCells + 1);
    int* CI = cell_idx + (size_t)f * cap;
    for (int c = tid; c <= kGridCells; c += 256) {  // lower_bound of cell c among the m valid keys
        const unsigned t = (unsigned)c << kGridKeyBits;
        int lo = 0, hi = m;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_key[mid] < t) lo = mid + 1;
            else hi = mid;
        }
        CO[c] = lo;
    }
    for (int j = tid; j < m; j += 256) CI[j] = (int)(s_key[j] & ((1u << kGridKeyBits) - 1));
}

struct ProjLds {
    float *kx, *ky;
    unsigned char *koct, *blocked, *pre, *nulled;
    int *cell_off, *assign, *best;
    unsigned short *cell_idx, *ent;
};

// GetFeaturesInArea + the candidate loop of SearchByProjection (:1992-2058)
// for LastFrame point i against the blocked flags `blk`; returns
// (bestDist << 16 | bestIdx2), or 0xFFFFFFFF when the point is skipped.
__device__ unsigned proj_scan(const plvi_proj_params& p, const ProjLds& s, const unsigned char* blk, int i,
                              const float* __restrict__ x3dc, const int* __restrict__ loct,
                              const uint8_t* __restrict__ mpdesc, const uint8_t* __restrict__ cdesc,
                              const float* __restrict__ uright, int n_cur) {
    const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
    const float invzc = (float)(1.0 / (double)zc);
    if (invzc < 0) return 0xFFFFFFFFu;
    const float u = p.fx * xc / zc + p.cx, v = p.fy * yc / zc + p.cy;  // Pinhole::project
    if (u < p.min_x || u > p.max_x) return 0xFFFFFFFFu;
    if (v < p.min_y || v > p.max_y) return 0xFFFFFFFFu;
    const int nLastOctave = loct[i];
    if (nLastOctave < 0 || nLastOctave >= p.nlevels) return 0xFFFFFFFFu;  // no scale factor: no candidate
    const float radius = p.th * p.scale_factors[nLastOctave];
    int minLevel, maxLevel;
    if (p.forward) { minLevel = nLastOctave; maxLevel = -1; }
    else if (p.backward) { minLevel = 0; maxLevel = nLastOctave; }
    else { minLevel = nLastOctave - 1; maxLevel = nLastOctave + 1; }
    const int nMinCellX = max(0, (int)floorf((u - p.min_x - radius) * p.inv_w));
    if (nMinCellX >= kGridCols) return 0xFFFFFFFFu;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((u - p.min_x + radius) * p.inv_w));
    if (nMaxCellX < 0) return 0xFFFFFFFFu;
    const int nMinCellY = max(0, (int)floorf((v - p.min_y - radius) * p.inv_h));
    if (nMinCellY >= kGridRows) return 0xFFFFFFFFu;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((v - p.min_y + radius) * p.inv_h));
    if (nMaxCellY < 0) return 0xFFFFFFFFu;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const uint4* dm = reinterpret_cast<const uint4*>(mpdesc + (size_t)32 * i);
    const uint4 m0 = dm[0], m1 = dm[1];
    int bestDist = 256, bestIdx2 = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int k0 = s.cell_off[ix * kGridRows + nMinCellY], k1 = s.cell_off[ix * kGridRows + nMaxCellY + 1];
        for (int k = k0; k < k1; ++k) {
            const int i2 = s.cell_idx[k];
            if (bCheckLevels) {
                const int o = s.koct[i2];
                if (o < minLevel) continue;
                if (maxLevel >= 0 && o > maxLevel) continue;
            }
            const float distx = s.kx[i2] - u, disty = s.ky[i2] - v;
            if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
            if (blk[i2]) continue;
            if (uright && uright[i2] > 0) {
                const float ur = rfmaf(-p.mbf, invzc, u);  // fused in ORBmatcher.cc.o
                const float er = fabsf(ur - uright[i2]);
                if (er > radius) continue;
            }
            const uint4* dc = reinterpret_cast<const uint4*>(cdesc + (size_t)32 * i2);
            const uint4 c0 = dc[0], c1 = dc[1];
            const int dist = __popc(m0.x ^ c0.x) + __popc(m0.y ^ c0.y) + __popc(m0.z ^ c0.z) + __popc(m0.w ^ c0.w) +
                             __popc(m1.x ^ c1.x) + __popc(m1.y ^ c1.y) + __popc(m1.z ^ c1.z) + __popc(m1.w ^ c1.w);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
    }
    if (bestIdx2 < 0) return 0xFFFFFFFFu;
    return ((unsigned)bestDist << 16) | (unsigned)bestIdx2;
}

__global__ __launch_bounds__(256) void search_by_projection_kernel(
    plvi_proj_params p, const plvi_keypoint* __restrict__ ckps, const uint8_t* __restrict__ cdesc_all,
    const int* __restrict__ cur_n, int cur_cap, const uint8_t* __restrict__ cblocked, const float* __restrict__ curight,
    const int* __restrict__ cell_off_all, const int* __restrict__ cell_idx_all, const float* __restrict__ x3dc_all,
    const int* __restrict__ loct_all, const float* __restrict__ lang_all, const uint8_t* __restrict__ mpdesc_all,
    const uint8_t* __restrict__ lflags_all, const int* __restrict__ last_n, int last_cap, int* __restrict__ match,
    int* __restrict__ nmatches) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int pr = blockIdx.x, tid = threadIdx.x;
    const int nc = min(cur_n[pr], cur_cap), nl = min(last_n[pr], last_cap);
    ProjLds s;
    {
        unsigned char* q = lds;
        s.kx = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.ky = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.assign = reinterpret_cast<int*>(q); q += 4 * cur_cap;
        s.best = reinterpret_cast<int*>(q); q += 4 * last_cap;
        s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kGridCells + 1);
        s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * cur_cap;
        s.ent = reinterpret_cast<unsigned short*>(q); q += 4 * last_cap;  // [last_cap] idx, [last_cap] bin
        s.koct = q; q += cur_cap;
        s.blocked = q; q += cur_cap;
        s.pre = q; q += cur_cap;
        s.nulled = q;
    }
    __shared__ int s_hist[kProjHisto], s_keep[3], s_ne, s_nm;
    const plvi_keypoint* K = ckps + (size_t)pr * cur_cap;
    const uint8_t* cdesc = cdesc_all + (size_t)pr * cur_cap * 32;
    const float* ur = curight ? curight + (size_t)pr * cur_cap : nullptr;
    for (int i = tid; i < nc; i += 256) {
        s.kx[i] = K[i].x;
        s.ky[i] = K[i].y;
        s.koct[i] = (unsigned char)K[i].octave;
        const unsigned char b = cblocked ? cblocked[(size_t)pr * cur_cap + i] : 0;
        s.blocked[i] = b;
        s.pre[i] = b;
        s.nulled[i] = 0;
        s.assign[i] = -1;
    }
    const int* CO = cell_off_all + (size_t)pr * (kGridCells + 1);
    for (int c = tid; c <= kGridCells; c += 256) s.cell_off[c] = CO[c];
    const int ncell = CO[kGridCells];
    for (int k = tid; k < ncell; k += 256) s.cell_idx[k] = (unsigned short)cell_idx_all[(size_t)pr * cur_cap + k];
    if (tid < kProjHisto) s_hist[tid] = 0;
    __syncthreads();
    const float* x3dc = x3dc_all + (size_t)pr * last_cap * 3;
    const int* loct = loct_all + (size_t)pr * last_cap;
    const uint8_t* mpdesc = mpdesc_all + (size_t)pr * last_cap * 32;
    const uint8_t* lflags = lflags_all + (size_t)pr * last_cap;
    // phase 1: every point against the flags on entry
    for (int i = tid; i < nl; i += 256)
        s.best[i] = (lflags[i] & 1) ? (int)proj_scan(p, s, s.pre, i, x3dc, loct, mpdesc, cdesc, ur, nc) : -1;
    __syncthreads();
    // phase 2: the greedy assignment in LastFrame order (:2060-2083)
    if (tid == 0) {
        const float factor = 1.0f / kProjHisto;
        const float* lang = lang_all + (size_t)pr * last_cap;
        int nm = 0, ne = 0;
        for (int i = 0; i < nl; ++i) {
            unsigned b = (unsigned)s.best[i];
            if (b == 0xFFFFFFFFu) continue;
            if (s.blocked[b & 0xFFFFu] != s.pre[b & 0xFFFFu])  // its best was taken meanwhile: re-scan
                b = proj_scan(p, s, s.blocked, i, x3dc, loct, mpdesc, cdesc, ur, nc);
            if (b == 0xFFFFFFFFu || (int)(b >> 16) > kProjThHigh) continue;
            const int i2 = (int)(b & 0xFFFFu);
            s.assign[i2] = i;
            s.blocked[i2] = (lflags[i] & 2) ? 1 : 0;  // the stored MapPoint's Observations() > 0
            ++nm;
            if (p.check_orientation) {
                float rot = lang[i] - K[i2].angle;
                if (rot < 0.0f) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == kProjHisto) bin = 0;
                s.ent[last_cap + ne] = (unsigned short)bin;
                s.ent[ne++] = (unsigned short)i2;
                s_hist[bin]++;
            }
        }
        s_ne = ne;
        s_nm = nm;
        // ComputeThreeMaxima (:2304-2345)
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int b = 0; b < kProjHisto; b++) {
            const int c = s_hist[b];
            if (c > max1) {
                max3 = max2; max2 = max1; max1 = c;
                ind3 = ind2; ind2 = ind1; ind1 = b;
            } else if (c > max2) {
                max3 = max2; max2 = c;
                ind3 = ind2; ind2 = b;
            } else if (c > max3) {
                max3 = c;
                ind3 = b;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        s_keep[0] = ind1; s_keep[1] = ind2; s_keep[2] = ind3;
    }
    __syncthreads();
    // phase 3: entries in dropped bins set mvpMapPoints[idx] = NULL (:2164-2174)
    if (p.check_orientation) {
        const int ne = s_ne;
        int dropped = 0;
        for (int e = tid; e < ne; e += 256) {
            const int bin = s.ent[last_cap + e];
            if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2]) {
                s.nulled[s.ent[e]] = 1;
                ++dropped;
            }
        }
        if (dropped) atomicSub(&s_nm, dropped);
        __syncthreads();
    }
    int* M = match + (size_t)pr * cur_cap;
    for (int i = tid; i < nc; i += 256) M[i] = s.nulled[i] ? -2 : s.assign[i];
    if (tid == 0) nmatches[pr] = s_nm;
}

// ---------------------------------------------------------------------------
// SearchByProjection(CurrentFrame, LastFrame, th, bMono) on a two-camera
// CurrentFrame (CurrentFrame.Nleft != -1, :1985-2153): every LastFrame point
// is projected with CurrentFrame.mpCamera into the left image (x3Dc) and,
// when the left pass did not `continue` (:2000-2026: behind the camera,
// outside the image bounds, empty window), into the right image (x3Dr =
// mTrl * x3Dc, no bounds test, mGridRight); no mvuRight test.  Both
// assignments feed one rotation histogram (right entries at idx + Nleft).
// mpCamera is Pinhole (:30-33) or KannalaBrandt8 (:33-48 of
// CameraModels/KannalaBrandt8.cpp, glibc atan2f / cosf / sinf restated in
// plvi_math.h).  Same schedule as the one-camera kernel, per side.
struct CamModel {
    int kb;  // 0 = Pinhole, 1 = KannalaBrandt8 (k1..k4 below)
    float k0, k1, k2, k3;
};

__device__ __forceinline__ void cam_project(const plvi_proj_params& p, const CamModel& cm, float x, float y, float z,
                                            float& u, float& v) {
    if (!cm.kb) {  // Pinhole::project
        u = p.fx * x / z + p.cx;
        v = p.fy * y / z + p.cy;
        return;
    }
    // KannalaBrandt8::project(const cv::Point3f&); its 7 fused multiply-adds
    // as in KannalaBrandt8.cpp.o (x*x + y*y, the four r terms, u, v)
    const float x2_plus_y2 = rfmaf(x, x, y * y);
    const float theta = plvi::plvi_atan2f(__builtin_sqrtf(x2_plus_y2), z);
    const float psi = plvi::plvi_atan2f(y, x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = rfmaf(cm.k3, theta9, rfmaf(cm.k2, theta7, rfmaf(cm.k1, theta5, rfmaf(cm.k0, theta3, theta))));
    u = rfmaf(p.fx * r, plvi::plvi_cosf(psi), p.cx);
    v = rfmaf(p.fy * r, plvi::plvi_sinf(psi), p.cy);
}

constexpr unsigned kScanSkip = 0xFFFFFFFFu;   // left pass `continue`d: no right pass either
constexpr unsigned kScanNone = 0xFFFFFFFEu;   // window searched, no candidate (bestIdx2 == -1)

// GetFeaturesInArea(u, v, radius, levels, bRight) + the candidate loop
// (:2033-2058 / :2109-2125) of point i on one side.
__device__ unsigned proj2_scan(const plvi_proj_params& p, const ProjLds& s, const unsigned char* blk, float u, float v,
                               int nLastOctave, const uint8_t* __restrict__ mpd, const uint8_t* __restrict__ cdesc,
                               bool left) {
    if (nLastOctave < 0 || nLastOctave >= p.nlevels) return left ? kScanSkip : kScanNone;  // no scale factor
    const float radius = p.th * p.scale_factors[nLastOctave];
    int minLevel, maxLevel;
    if (p.forward) { minLevel = nLastOctave; maxLevel = -1; }
    else if (p.backward) { minLevel = 0; maxLevel = nLastOctave; }
    else { minLevel = nLastOctave - 1; maxLevel = nLastOctave + 1; }
    const unsigned empty = left ? kScanSkip : kScanNone;
    const int nMinCellX = max(0, (int)floorf((u - p.min_x - radius) * p.inv_w));
    if (nMinCellX >= kGridCols) return empty;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((u - p.min_x + radius) * p.inv_w));
    if (nMaxCellX < 0) return empty;
    const int nMinCellY = max(0, (int)floorf((v - p.min_y - radius) * p.inv_h));
    if (nMinCellY >= kGridRows) return empty;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((v - p.min_y + radius) * p.inv_h));
    if (nMaxCellY < 0) return empty;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const uint4* dm = reinterpret_cast<const uint4*>(mpd);
    const uint4 m0 = dm[0], m1 = dm[1];
    int bestDist = 256, bestIdx2 = -1;
    bool any = false;  // vIndices2 non-empty
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int k0 = s.cell_off[ix * kGridRows + nMinCellY], k1 = s.cell_off[ix * kGridRows + nMaxCellY + 1];
        for (int k = k0; k < k1; ++k) {
            const int i2 = s.cell_idx[k];
            if (bCheckLevels) {
                const int o = s.koct[i2];
                if (o < minLevel) continue;
                if (maxLevel >= 0 && o > maxLevel) continue;
            }
            const float distx = s.kx[i2] - u, disty = s.ky[i2] - v;
            if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
            any = true;
            if (blk[i2]) continue;
            const uint4* dc = reinterpret_cast<const uint4*>(cdesc + (size_t)32 * i2);
            const uint4 c0 = dc[0], c1 = dc[1];
            const int dist = __popc(m0.x ^ c0.x) + __popc(m0.y ^ c0.y) + __popc(m0.z ^ c0.z) + __popc(m0.w ^ c0.w) +
                             __popc(m1.x ^ c1.x) + __popc(m1.y ^ c1.y) + __popc(m1.z ^ c1.z) + __popc(m1.w ^ c1.w);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
    }
    if (!any) return empty;
    if (bestIdx2 < 0) return kScanNone;
    return ((unsigned)bestDist << 16) | (unsigned)bestIdx2;
}

struct ProjSide {
    ProjLds s;
    const plvi_keypoint* K;
    const uint8_t* desc;
    int n;
};

__device__ void proj_side_load(ProjSide& d, unsigned char*& q, int cap, const uint8_t* blocked, const int* CO,
                               const int* CI, int tid) {
    d.s.kx = reinterpret_cast<float*>(q); q += 4 * cap;
    d.s.ky = reinterpret_cast<float*>(q); q += 4 * cap;
    d.s.assign = reinterpret_cast<int*>(q); q += 4 * cap;
    d.s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kGridCells + 1);
    d.s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * cap;
    d.s.koct = q; q += cap;
    d.s.blocked = q; q += cap;
    d.s.pre = q; q += cap;
    d.s.nulled = q; q += cap;
    q = reinterpret_cast<unsigned char*>(((uintptr_t)q + 15) & ~(uintptr_t)15);
    for (int i = tid; i < d.n; i += 256) {
        d.s.kx[i] = d.K[i].x;
        d.s.ky[i] = d.K[i].y;
        d.s.koct[i] = (unsigned char)d.K[i].octave;
        const unsigned char b = blocked ? (blocked[i] != 0) : 0;
        d.s.blocked[i] = b;
        d.s.pre[i] = b;
        d.s.nulled[i] = 0;
        d.s.assign[i] = -1;
    }
    for (int c = tid; c <= kGridCells; c += 256) d.s.cell_off[c] = CO[c];
    const int ncell = CO[kGridCells];
    for (int k = tid; k < ncell; k += 256) d.s.cell_idx[k] = (unsigned short)CI[k];
}

__global__ __launch_bounds__(256) void search_by_projection2_kernel(
    plvi_proj_params p, CamModel cm, const plvi_keypoint* __restrict__ lkps, const uint8_t* __restrict__ ldesc_all,
    const int* __restrict__ l_n, int l_cap, const uint8_t* __restrict__ lblocked, const int* __restrict__ lcell_off_all,
    const int* __restrict__ lcell_idx_all, const plvi_keypoint* __restrict__ rkps, const uint8_t* __restrict__ rdesc_all,
    const int* __restrict__ r_n, int r_cap, const uint8_t* __restrict__ rblocked, const int* __restrict__ rcell_off_all,
    const int* __restrict__ rcell_idx_all, const float* __restrict__ x3dc_all, const float* __restrict__ x3dr_all,
    const int* __restrict__ loct_all, const float* __restrict__ lang_all, const uint8_t* __restrict__ mpdesc_all,
    const uint8_t* __restrict__ lflags_all, const int* __restrict__ last_n, int last_cap, int* __restrict__ match_l,
    int* __restrict__ match_r, int* __restrict__ nmatches) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int pr = blockIdx.x, tid = threadIdx.x;
    const int nl = min(last_n[pr], last_cap);
    ProjSide S[2];
    S[0].n = min(l_n[pr], l_cap);
    S[1].n = min(r_n[pr], r_cap);
    S[0].K = lkps + (size_t)pr * l_cap;
    S[1].K = rkps + (size_t)pr * r_cap;
    S[0].desc = ldesc_all + (size_t)pr * l_cap * 32;
    S[1].desc = rdesc_all + (size_t)pr * r_cap * 32;
    unsigned* best;          // [2][last_cap]
    unsigned short* ent;     // [2 * last_cap] keypoint, [2 * last_cap] bin | side << 15
    {
        unsigned char* q = lds;
        best = reinterpret_cast<unsigned*>(q); q += 8 * (size_t)last_cap;
        ent = reinterpret_cast<unsigned short*>(q); q += 8 * (size_t)last_cap;
        proj_side_load(S[0], q, l_cap, lblocked ? lblocked + (size_t)pr * l_cap : nullptr,
                       lcell_off_all + (size_t)pr * (kGridCells + 1), lcell_idx_all + (size_t)pr * l_cap, tid);
        proj_side_load(S[1], q, r_cap, rblocked ? rblocked + (size_t)pr * r_cap : nullptr,
                       rcell_off_all + (size_t)pr * (kGridCells + 1), rcell_idx_all + (size_t)pr * r_cap, tid);
    }
    __shared__ int s_hist[kProjHisto], s_keep[3], s_ne, s_nm;
    if (tid < kProjHisto) s_hist[tid] = 0;
    __syncthreads();
    const float* x3dc = x3dc_all + (size_t)pr * last_cap * 3;
    const float* x3dr = x3dr_all + (size_t)pr * last_cap * 3;
    const int* loct = loct_all + (size_t)pr * last_cap;
    const uint8_t* mpdesc = mpdesc_all + (size_t)pr * last_cap * 32;
    const uint8_t* lflags = lflags_all + (size_t)pr * last_cap;
    // the projections of point i (left pass exits: invzc < 0, outside the bounds)
    auto project = [&](int i, float& ul, float& vl, float& ur, float& vr) -> bool {
        const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
        const float invzc = (float)(1.0 / (double)zc);
        if (invzc < 0) return false;
        cam_project(p, cm, xc, yc, zc, ul, vl);
        if (ul < p.min_x || ul > p.max_x) return false;
        if (vl < p.min_y || vl > p.max_y) return false;
        cam_project(p, cm, x3dr[3 * i], x3dr[3 * i + 1], x3dr[3 * i + 2], ur, vr);
        return true;
    };
    // phase 1: both sides of every point against the flags on entry
    for (int i = tid; i < nl; i += 256) {
        unsigned bl = kScanSkip, br = kScanSkip;
        float ul, vl, ur, vr;
        if ((lflags[i] & 1) && project(i, ul, vl, ur, vr)) {
            const uint8_t* mpd = mpdesc + (size_t)32 * i;
            bl = proj2_scan(p, S[0].s, S[0].s.pre, ul, vl, loct[i], mpd, S[0].desc, true);
            if (bl != kScanSkip) br = proj2_scan(p, S[1].s, S[1].s.pre, ur, vr, loct[i], mpd, S[1].desc, false);
        }
        best[i] = bl;
        best[last_cap + i] = br;
    }
    __syncthreads();
    // phase 2: LastFrame order, left (:2060-2083) then right (:2127-2148)
    if (tid == 0) {
        const float factor = 1.0f / kProjHisto;
        const float* lang = lang_all + (size_t)pr * last_cap;
        int nm = 0, ne = 0;
        for (int i = 0; i < nl; ++i) {
            if (best[i] == kScanSkip) continue;
            float ul, vl, ur, vr;
            bool projected = false;
            for (int c = 0; c < 2; ++c) {
                ProjSide& A = S[c];
                unsigned b = best[c * last_cap + i];
                if (b == kScanSkip || b == kScanNone) continue;  // no unblocked candidate stays so
                if (A.s.blocked[b & 0xFFFFu] != A.s.pre[b & 0xFFFFu]) {  // its best was taken meanwhile: re-scan
                    if (!projected) projected = project(i, ul, vl, ur, vr);
                    b = proj2_scan(p, A.s, A.s.blocked, c ? ur : ul, c ? vr : vl, loct[i], mpdesc + (size_t)32 * i,
                                   A.desc, c == 0);
                    if (b == kScanSkip || b == kScanNone) continue;
                }
                if ((int)(b >> 16) > kProjThHigh) continue;
                const int i2 = (int)(b & 0xFFFFu);
                A.s.assign[i2] = i;
                A.s.blocked[i2] = (lflags[i] & 2) ? 1 : 0;  // the stored MapPoint's Observations() > 0
                ++nm;
                if (p.check_orientation) {
                    float rot = lang[i] - A.K[i2].angle;
                    if (rot < 0.0f) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == kProjHisto) bin = 0;
                    ent[2 * last_cap + ne] = (unsigned short)(bin | c << 15);
                    ent[ne++] = (unsigned short)i2;
                    s_hist[bin]++;
                }
            }
        }
        s_ne = ne;
        s_nm = nm;
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;  // ComputeThreeMaxima (:2304-2345)
        for (int b = 0; b < kProjHisto; b++) {
            const int c = s_hist[b];
            if (c > max1) {
                max3 = max2; max2 = max1; max1 = c;
                ind3 = ind2; ind2 = ind1; ind1 = b;
            } else if (c > max2) {
                max3 = max2; max2 = c;
                ind3 = ind2; ind2 = b;
            } else if (c > max3) {
                max3 = c;
                ind3 = b;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        s_keep[0] = ind1; s_keep[1] = ind2; s_keep[2] = ind3;
    }
    __syncthreads();
    // phase 3: entries in dropped bins set mvpMapPoints[idx] = NULL (:2155-2175)
    if (p.check_orientation) {
        const int ne = s_ne;
        int dropped = 0;
        for (int e = tid; e < ne; e += 256) {
            const int code = ent[2 * last_cap + e], bin = code & 0x7FFF;
            if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2]) {
                S[code >> 15].s.nulled[ent[e]] = 1;
                ++dropped;
            }
        }
        if (dropped) atomicSub(&s_nm, dropped);
        __syncthreads();
    }
    int* ML = match_l + (size_t)pr * l_cap;
    int* MR = match_r + (size_t)pr * r_cap;
    for (int i = tid; i < S[0].n; i += 256) ML[i] = S[0].s.nulled[i] ? -2 : S[0].s.assign[i];
    for (int i = tid; i < S[1].n; i += 256) MR[i] = S[1].s.nulled[i] ? -2 : S[1].s.assign[i];
    if (tid == 0) nmatches[pr] = s_nm;
}

// ---------------------------------------------------------------------------
// ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th,
// bFarPoints, thFarPoints) (src/ORBmatcher.cc:44-145, F.Nleft == -1): the
// local-map search of Tracking::SearchLocalPoints (Tracking.cc:5119/5211).
// Same schedule as above: phase 1 scans every MapPoint's window in parallel
// against the flags on entry and keeps its best and second candidate
// (first argmin, then first argmin of the rest -- the scan order of
// GetFeaturesInArea); phase 2 walks the MapPoints in vector order and
// re-scans only one whose best or second candidate was blocked meanwhile
// (removing any other candidate leaves both unchanged), then applies the
// level-aware ratio test and the assignment.
// fbit: the MapPoint flag that enables this scan; use_th: the radius is
// scaled by th (the left camera's branch only, :69-70 -- not :148)
__device__ void local_scan(const plvi_local_params& p, const ProjLds& s, const unsigned char* blk, int m,
                           const unsigned char* __restrict__ fl, const float* __restrict__ proj,
                           const int* __restrict__ lvl, const uint8_t* __restrict__ mpdesc,
                           const uint8_t* __restrict__ cdesc, const float* __restrict__ uright, unsigned* b1,
                           unsigned* b2, unsigned char fbit = 1, bool use_th = true) {
    *b1 = *b2 = 0xFFFFFFFFu;
    if (!(fl[m] & fbit)) return;
    const float x = proj[4 * m], y = proj[4 * m + 1], xr = proj[4 * m + 2], vcos = proj[4 * m + 3];
    const int L = lvl[m];
    if (L < 0 || L >= p.nlevels) return;  // no scale factor for that level: no candidate
    float r = vcos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:216-222)
    if (use_th && p.th != 1.0) r *= p.th;
    const float radius = r * p.scale_factors[L];
    const int minLevel = L - 1, maxLevel = L;
    const int nMinCellX = max(0, (int)floorf((x - p.min_x - radius) * p.inv_w));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - p.min_x + radius) * p.inv_w));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - p.min_y - radius) * p.inv_h));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - p.min_y + radius) * p.inv_h));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const uint4* dm = reinterpret_cast<const uint4*>(mpdesc + (size_t)32 * m);
    const uint4 m0 = dm[0], m1 = dm[1];
    int bestDist = 256, bestDist2 = 256, bestIdx = -1, secondIdx = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int k0 = s.cell_off[ix * kGridRows + nMinCellY], k1 = s.cell_off[ix * kGridRows + nMaxCellY + 1];
        for (int k = k0; k < k1; ++k) {
            const int idx = s.cell_idx[k];
            if (bCheckLevels) {
                const int o = s.koct[idx];
                if (o < minLevel) continue;
                if (maxLevel >= 0 && o > maxLevel) continue;
            }
            const float distx = s.kx[idx] - x, disty = s.ky[idx] - y;
            if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
            if (blk[idx]) continue;
            if (uright && uright[idx] > 0) {
                const float er = fabsf(xr - uright[idx]);
                if (er > radius) continue;
            }
            const uint4* dc = reinterpret_cast<const uint4*>(cdesc + (size_t)32 * idx);
            const uint4 c0 = dc[0], c1 = dc[1];
            const int dist = __popc(m0.x ^ c0.x) + __popc(m0.y ^ c0.y) + __popc(m0.z ^ c0.z) + __popc(m0.w ^ c0.w) +
                             __popc(m1.x ^ c1.x) + __popc(m1.y ^ c1.y) + __popc(m1.z ^ c1.z) + __popc(m1.w ^ c1.w);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                secondIdx = bestIdx;
                bestDist = dist;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
                secondIdx = idx;
            }
        }
    }
    if (bestIdx < 0) return;
    *b1 = ((unsigned)bestDist << 16) | (unsigned)bestIdx;
    if (secondIdx >= 0) *b2 = ((unsigned)bestDist2 << 16) | (unsigned)secondIdx;
}

__global__ __launch_bounds__(256) void search_local_kernel(
    plvi_local_params p, const plvi_keypoint* __restrict__ ckps, const uint8_t* __restrict__ cdesc_all,
    const int* __restrict__ cur_n, int cur_cap, const uint8_t* __restrict__ cblocked, const float* __restrict__ curight,
    const int* __restrict__ cell_off_all, const int* __restrict__ cell_idx_all, const uint8_t* __restrict__ flags_all,
    const float* __restrict__ proj_all, const int* __restrict__ level_all, const uint8_t* __restrict__ mpdesc_all,
    const int* __restrict__ mp_n, int mp_cap, int* __restrict__ match, int* __restrict__ nmatches) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int fr = blockIdx.x, tid = threadIdx.x;
    const int nc = min(cur_n[fr], cur_cap), nm = min(mp_n[fr], mp_cap);
    ProjLds s;
    unsigned *best1, *best2;
    {
        unsigned char* q = lds;
        s.kx = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.ky = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.assign = reinterpret_cast<int*>(q); q += 4 * cur_cap;
        best1 = reinterpret_cast<unsigned*>(q); q += 4 * mp_cap;
        best2 = reinterpret_cast<unsigned*>(q); q += 4 * mp_cap;
        s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kGridCells + 1);
        s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * cur_cap;
        s.koct = q; q += cur_cap;
        s.blocked = q; q += cur_cap;
        s.pre = q;
    }
    const plvi_keypoint* K = ckps + (size_t)fr * cur_cap;
    const uint8_t* cdesc = cdesc_all + (size_t)fr * cur_cap * 32;
    const float* ur = curight ? curight + (size_t)fr * cur_cap : nullptr;
    for (int i = tid; i < nc; i += 256) {
        s.kx[i] = K[i].x;
        s.ky[i] = K[i].y;
        s.koct[i] = (unsigned char)K[i].octave;
        const unsigned char b = cblocked ? cblocked[(size_t)fr * cur_cap + i] : 0;
        s.blocked[i] = b;
        s.pre[i] = b;
        s.assign[i] = -1;
    }
    const int* CO = cell_off_all + (size_t)fr * (kGridCells + 1);
    for (int c = tid; c <= kGridCells; c += 256) s.cell_off[c] = CO[c];
    const int ncell = CO[kGridCells];
    for (int k = tid; k < ncell; k += 256) s.cell_idx[k] = (unsigned short)cell_idx_all[(size_t)fr * cur_cap + k];
    __syncthreads();
    const unsigned char* fl = flags_all + (size_t)fr * mp_cap;
    const float* proj = proj_all + (size_t)fr * mp_cap * 4;
    const int* lvl = level_all + (size_t)fr * mp_cap;
    const uint8_t* mpdesc = mpdesc_all + (size_t)fr * mp_cap * 32;
    // phase 1: every MapPoint against the flags on entry
    for (int m = tid; m < nm; m += 256) local_scan(p, s, s.pre, m, fl, proj, lvl, mpdesc, cdesc, ur, &best1[m], &best2[m]);
    __syncthreads();
    // phase 2: the assignment in vpMapPoints order (:98-117)
    if (tid == 0) {
        int nmt = 0;
        for (int m = 0; m < nm; ++m) {
            unsigned b1 = best1[m], b2 = best2[m];
            if (b1 == 0xFFFFFFFFu) continue;
            const int i1 = (int)(b1 & 0xFFFFu), i2 = b2 == 0xFFFFFFFFu ? -1 : (int)(b2 & 0xFFFFu);
            if (s.blocked[i1] != s.pre[i1] || (i2 >= 0 && s.blocked[i2] != s.pre[i2])) {
                local_scan(p, s, s.blocked, m, fl, proj, lvl, mpdesc, cdesc, ur, &b1, &b2);  // blocked meanwhile
                if (b1 == 0xFFFFFFFFu) continue;
            }
            const int bestDist = (int)(b1 >> 16), bestIdx = (int)(b1 & 0xFFFFu);
            const int bestDist2 = b2 == 0xFFFFFFFFu ? 256 : (int)(b2 >> 16);
            const int bestLevel = s.koct[bestIdx], bestLevel2 = b2 == 0xFFFFFFFFu ? -1 : s.koct[b2 & 0xFFFFu];
            if (bestDist <= kProjThHigh) {
                if (bestLevel == bestLevel2 && bestDist > p.nnratio * bestDist2) continue;
                if (bestLevel != bestLevel2 || bestDist <= p.nnratio * bestDist2) {
                    s.assign[bestIdx] = m;
                    s.blocked[bestIdx] = (fl[m] & 2) ? 1 : 0;  // the stored MapPoint's Observations() > 0
                    ++nmt;
                }
            }
        }
        nmatches[fr] = nmt;
    }
    __syncthreads();
    int* M = match + (size_t)fr * cur_cap;
    for (int i = tid; i < nc; i += 256) M[i] = s.assign[i];
}

// ---------------------------------------------------------------------------
// The same search on a two-camera Frame (F.Nleft != -1: the KannalaBrandt8
// stereo rigs, ORBmatcher.cc:44-214).  Left keypoints mvKeys [0, Nleft) with
// grid mGrid, right keypoints mvKeysRight with mGridRight (right-relative
// indices, Frame.cc:661-674); a MapPoint is searched in the left image when
// mbTrackInView (flag bit0) and in the right image when mbTrackInViewR (bit2)
// -- the right radius is not scaled by th (:148) and there is no mvuRight
// test.  Assignments follow the stereo pairs: a left match also stores the
// MapPoint at mvLeftToRightMatch[idx] + Nleft (:132-136), a right match at
// mvRightToLeftMatch[idx] (:199-203), and both block those keypoints for the
// later MapPoints.  A left ratio-test failure skips the MapPoint's right
// search too (the `continue` at :127).  Same schedule: phase 1 scans both
// sides of every MapPoint in parallel against the entry flags, phase 2 walks
// the MapPoints in order, left then right, re-scanning a side whose best or
// second candidate was blocked meanwhile.
struct LocalSide {
    ProjLds s;
    const uint8_t* desc;
    const int* pair;  // mvLeftToRightMatch / mvRightToLeftMatch (NULL = none)
    int n;
};

__device__ void local_side_load(LocalSide& d, unsigned char*& q, int cap, const plvi_keypoint* K,
                                const uint8_t* blocked, const int* CO, const int* CI, int tid) {
    d.s.kx = reinterpret_cast<float*>(q); q += 4 * cap;
    d.s.ky = reinterpret_cast<float*>(q); q += 4 * cap;
    d.s.assign = reinterpret_cast<int*>(q); q += 4 * cap;
    d.s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kGridCells + 1);
    d.s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * cap;
    d.s.koct = q; q += cap;
    d.s.blocked = q; q += cap;
    d.s.pre = q; q += cap;
    q = reinterpret_cast<unsigned char*>(((uintptr_t)q + 15) & ~(uintptr_t)15);
    for (int i = tid; i < d.n; i += 256) {
        d.s.kx[i] = K[i].x;
        d.s.ky[i] = K[i].y;
        d.s.koct[i] = (unsigned char)K[i].octave;
        const unsigned char b = blocked ? blocked[i] : 0;
        d.s.blocked[i] = b;
        d.s.pre[i] = b;
        d.s.assign[i] = -1;
    }
    for (int c = tid; c <= kGridCells; c += 256) d.s.cell_off[c] = CO[c];
    const int ncell = CO[kGridCells];
    for (int k = tid; k < ncell; k += 256) d.s.cell_idx[k] = (unsigned short)CI[k];
}

__global__ __launch_bounds__(256) void search_local2_kernel(
    plvi_local_params p, const plvi_keypoint* __restrict__ lkps, const uint8_t* __restrict__ ldesc_all,
    const int* __restrict__ l_n, int l_cap, const uint8_t* __restrict__ lblocked, const int* __restrict__ l2r_all,
    const int* __restrict__ lcell_off_all, const int* __restrict__ lcell_idx_all, const plvi_keypoint* __restrict__ rkps,
    const uint8_t* __restrict__ rdesc_all, const int* __restrict__ r_n, int r_cap, const uint8_t* __restrict__ rblocked,
    const int* __restrict__ r2l_all, const int* __restrict__ rcell_off_all, const int* __restrict__ rcell_idx_all,
    const uint8_t* __restrict__ flags_all, const float* __restrict__ proj_all, const int* __restrict__ level_all,
    const float* __restrict__ projr_all, const int* __restrict__ levelr_all, const uint8_t* __restrict__ mpdesc_all,
    const int* __restrict__ mp_n, int mp_cap, int* __restrict__ match_l, int* __restrict__ match_r,
    int* __restrict__ nmatches) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int fr = blockIdx.x, tid = threadIdx.x;
    const int nm = min(mp_n[fr], mp_cap);
    LocalSide S[2];
    S[0].n = min(l_n[fr], l_cap);
    S[1].n = min(r_n[fr], r_cap);
    S[0].desc = ldesc_all + (size_t)fr * l_cap * 32;
    S[1].desc = rdesc_all + (size_t)fr * r_cap * 32;
    S[0].pair = l2r_all ? l2r_all + (size_t)fr * l_cap : nullptr;
    S[1].pair = r2l_all ? r2l_all + (size_t)fr * r_cap : nullptr;
    unsigned* best;  // [4][mp_cap]: left best / second, right best / second
    {
        unsigned char* q = lds;
        best = reinterpret_cast<unsigned*>(q); q += 16 * (size_t)mp_cap;
        local_side_load(S[0], q, l_cap, lkps + (size_t)fr * l_cap, lblocked ? lblocked + (size_t)fr * l_cap : nullptr,
                        lcell_off_all + (size_t)fr * (kGridCells + 1), lcell_idx_all + (size_t)fr * l_cap, tid);
        local_side_load(S[1], q, r_cap, rkps + (size_t)fr * r_cap, rblocked ? rblocked + (size_t)fr * r_cap : nullptr,
                        rcell_off_all + (size_t)fr * (kGridCells + 1), rcell_idx_all + (size_t)fr * r_cap, tid);
    }
    __syncthreads();
    const unsigned char* fl = flags_all + (size_t)fr * mp_cap;
    const float* proj[2] = {proj_all + (size_t)fr * mp_cap * 4, projr_all + (size_t)fr * mp_cap * 4};
    const int* lvl[2] = {level_all + (size_t)fr * mp_cap, levelr_all + (size_t)fr * mp_cap};
    const uint8_t* mpdesc = mpdesc_all + (size_t)fr * mp_cap * 32;
    const unsigned char fbit[2] = {1, 4};
    // phase 1: both sides of every MapPoint against the flags on entry
    for (int m = tid; m < nm; m += 256)
        for (int c = 0; c < 2; ++c)
            local_scan(p, S[c].s, S[c].s.pre, m, fl, proj[c], lvl[c], mpdesc, S[c].desc, nullptr,
                       &best[(2 * c) * mp_cap + m], &best[(2 * c + 1) * mp_cap + m], fbit[c], c == 0);
    __syncthreads();
    // phase 2: vpMapPoints order, left (:62-143) then right (:145-211)
    // A stereo partner is overwritten unchecked (:133, :200), so a keypoint
    // blocked on entry can become a candidate again (stored MapPoint without
    // observations): from then on every scan of that image is redone (rare).
    if (tid == 0) {
        int nmt = 0;
        bool unblocked[2] = {false, false};
        for (int m = 0; m < nm; ++m) {
            const unsigned char obs = (fl[m] & 2) ? 1 : 0;  // the stored MapPoint's Observations() > 0
            for (int c = 0; c < 2; ++c) {
                LocalSide& A = S[c];
                LocalSide& B = S[1 - c];
                unsigned b1 = best[(2 * c) * mp_cap + m], b2 = best[(2 * c + 1) * mp_cap + m];
                if (b1 == 0xFFFFFFFFu && !unblocked[c]) continue;
                const int i1 = (int)(b1 & 0xFFFFu), i2 = b2 == 0xFFFFFFFFu ? -1 : (int)(b2 & 0xFFFFu);
                if (unblocked[c] || A.s.blocked[i1] != A.s.pre[i1] || (i2 >= 0 && A.s.blocked[i2] != A.s.pre[i2])) {
                    local_scan(p, A.s, A.s.blocked, m, fl, proj[c], lvl[c], mpdesc, A.desc, nullptr, &b1, &b2, fbit[c],
                               c == 0);  // blocked meanwhile
                    if (b1 == 0xFFFFFFFFu) continue;
                }
                const int bestDist = (int)(b1 >> 16), bestIdx = (int)(b1 & 0xFFFFu);
                const int bestDist2 = b2 == 0xFFFFFFFFu ? 256 : (int)(b2 >> 16);
                const int bestLevel = A.s.koct[bestIdx], bestLevel2 = b2 == 0xFFFFFFFFu ? -1 : A.s.koct[b2 & 0xFFFFu];
                if (bestDist > kProjThHigh) continue;
                if (bestLevel == bestLevel2 && bestDist > p.nnratio * bestDist2) break;  // :127 / :197: next MapPoint
                A.s.assign[bestIdx] = m;
                A.s.blocked[bestIdx] = obs;
                ++nmt;
                const int o = A.pair ? A.pair[bestIdx] : -1;
                if (o >= 0 && o < B.n) {  // the stereo observation in the other image
                    B.s.assign[o] = m;
                    if (B.s.blocked[o] && !obs) unblocked[1 - c] = true;
                    B.s.blocked[o] = obs;
                    ++nmt;
                }
            }
        }
        nmatches[fr] = nmt;
    }
    __syncthreads();
    int* ML = match_l + (size_t)fr * l_cap;
    int* MR = match_r + (size_t)fr * r_cap;
    for (int i = tid; i < S[0].n; i += 256) ML[i] = S[0].s.assign[i];
    for (int i = tid; i < S[1].n; i += 256) MR[i] = S[1].s.assign[i];
}

// ---------------------------------------------------------------------------
// ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
// const set<MapPoint*>& sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:2180-2300),
// the relocalization guided search (Tracking.cc:5857, 5871).  Same schedule as
// the frame-to-frame matcher: phase 1 finds every KF MapPoint's best candidate
// in parallel against the NULL / non-NULL mvpMapPoints on entry; phase 2
// walks the MapPoints in KF order -- every assignment blocks its keypoint for
// the later points (:2240-2242), so a point whose best was taken meanwhile is
// re-scanned -- and phase 3 is the rotation filter.
__device__ unsigned reloc_scan(const plvi_reloc_params& p, const ProjLds& s, const unsigned char* blk, int i,
                               const float* __restrict__ x3dc, const float* __restrict__ dist,
                               const int* __restrict__ lvl, const uint8_t* __restrict__ mpdesc,
                               const uint8_t* __restrict__ cdesc) {
    const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
    const float u = p.fx * xc / zc + p.cx, v = p.fy * yc / zc + p.cy;  // Pinhole::project (no depth test here)
    if (u < p.min_x || u > p.max_x) return 0xFFFFFFFFu;
    if (v < p.min_y || v > p.max_y) return 0xFFFFFFFFu;
    const float dist3D = dist[3 * i], minDistance = dist[3 * i + 1], maxDistance = dist[3 * i + 2];
    if (dist3D < minDistance || dist3D > maxDistance) return 0xFFFFFFFFu;
    const int L = lvl[i];
    if (L < 0 || L >= p.nlevels) return 0xFFFFFFFFu;  // PredictScale clamps to [0, mnScaleLevels)
    const float radius = p.th * p.scale_factors[L];
    const int minLevel = L - 1, maxLevel = L + 1;
    const int nMinCellX = max(0, (int)floorf((u - p.min_x - radius) * p.inv_w));
    if (nMinCellX >= kGridCols) return 0xFFFFFFFFu;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((u - p.min_x + radius) * p.inv_w));
    if (nMaxCellX < 0) return 0xFFFFFFFFu;
    const int nMinCellY = max(0, (int)floorf((v - p.min_y - radius) * p.inv_h));
    if (nMinCellY >= kGridRows) return 0xFFFFFFFFu;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((v - p.min_y + radius) * p.inv_h));
    if (nMaxCellY < 0) return 0xFFFFFFFFu;
    const uint4* dm = reinterpret_cast<const uint4*>(mpdesc + (size_t)32 * i);
    const uint4 m0 = dm[0], m1 = dm[1];
    int bestDist = 256, bestIdx2 = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int k0 = s.cell_off[ix * kGridRows + nMinCellY], k1 = s.cell_off[ix * kGridRows + nMaxCellY + 1];
        for (int k = k0; k < k1; ++k) {
            const int i2 = s.cell_idx[k];
            const int o = s.koct[i2];  // bCheckLevels holds: maxLevel >= 0
            if (o < minLevel || o > maxLevel) continue;
            const float distx = s.kx[i2] - u, disty = s.ky[i2] - v;
            if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
            if (blk[i2]) continue;
            const uint4* dc = reinterpret_cast<const uint4*>(cdesc + (size_t)32 * i2);
            const uint4 c0 = dc[0], c1 = dc[1];
            const int d = __popc(m0.x ^ c0.x) + __popc(m0.y ^ c0.y) + __popc(m0.z ^ c0.z) + __popc(m0.w ^ c0.w) +
                          __popc(m1.x ^ c1.x) + __popc(m1.y ^ c1.y) + __popc(m1.z ^ c1.z) + __popc(m1.w ^ c1.w);
            if (d < bestDist) {
                bestDist = d;
                bestIdx2 = i2;
            }
        }
    }
    if (bestIdx2 < 0) return 0xFFFFFFFFu;
    return ((unsigned)bestDist << 16) | (unsigned)bestIdx2;
}

__global__ __launch_bounds__(256) void search_reloc_kernel(
    plvi_reloc_params p, const plvi_keypoint* __restrict__ ckps, const uint8_t* __restrict__ cdesc_all,
    const int* __restrict__ cur_n, int cur_cap, const uint8_t* __restrict__ cblocked,
    const int* __restrict__ cell_off_all, const int* __restrict__ cell_idx_all, const uint8_t* __restrict__ kflags_all,
    const float* __restrict__ x3dc_all, const float* __restrict__ dist_all, const int* __restrict__ lvl_all,
    const float* __restrict__ kang_all, const uint8_t* __restrict__ mpdesc_all, const int* __restrict__ kf_n,
    int kf_cap, int* __restrict__ match, int* __restrict__ nmatches) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int pr = blockIdx.x, tid = threadIdx.x;
    const int nc = min(cur_n[pr], cur_cap), nk = min(kf_n[pr], kf_cap);
    ProjLds s;
    {
        unsigned char* q = lds;
        s.kx = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.ky = reinterpret_cast<float*>(q); q += 4 * cur_cap;
        s.assign = reinterpret_cast<int*>(q); q += 4 * cur_cap;
        s.best = reinterpret_cast<int*>(q); q += 4 * kf_cap;
        s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kGridCells + 1);
        s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * cur_cap;
        s.ent = reinterpret_cast<unsigned short*>(q); q += 4 * kf_cap;  // [kf_cap] idx, [kf_cap] bin
        s.koct = q; q += cur_cap;
        s.blocked = q; q += cur_cap;
        s.pre = q; q += cur_cap;
        s.nulled = q;
    }
    __shared__ int s_hist[kProjHisto], s_keep[3], s_ne, s_nm;
    const plvi_keypoint* K = ckps + (size_t)pr * cur_cap;
    const uint8_t* cdesc = cdesc_all + (size_t)pr * cur_cap * 32;
    for (int i = tid; i < nc; i += 256) {
        s.kx[i] = K[i].x;
        s.ky[i] = K[i].y;
        s.koct[i] = (unsigned char)K[i].octave;
        const unsigned char b = cblocked ? (cblocked[(size_t)pr * cur_cap + i] != 0) : 0;
        s.blocked[i] = b;
        s.pre[i] = b;
        s.nulled[i] = 0;
        s.assign[i] = -1;
    }
    const int* CO = cell_off_all + (size_t)pr * (kGridCells + 1);
    for (int c = tid; c <= kGridCells; c += 256) s.cell_off[c] = CO[c];
    const int ncell = CO[kGridCells];
    for (int k = tid; k < ncell; k += 256) s.cell_idx[k] = (unsigned short)cell_idx_all[(size_t)pr * cur_cap + k];
    if (tid < kProjHisto) s_hist[tid] = 0;
    __syncthreads();
    const float* x3dc = x3dc_all + (size_t)pr * kf_cap * 3;
    const float* dist = dist_all + (size_t)pr * kf_cap * 3;
    const int* lvl = lvl_all + (size_t)pr * kf_cap;
    const uint8_t* mpdesc = mpdesc_all + (size_t)pr * kf_cap * 32;
    const uint8_t* kfl = kflags_all + (size_t)pr * kf_cap;
    // phase 1: every KF MapPoint against mvpMapPoints on entry
    for (int i = tid; i < nk; i += 256)
        s.best[i] = (kfl[i] & 1) ? (int)reloc_scan(p, s, s.pre, i, x3dc, dist, lvl, mpdesc, cdesc) : -1;
    __syncthreads();
    // phase 2: the assignment in KF order (:2260-2277)
    if (tid == 0) {
        const float factor = 1.0f / kProjHisto;
        const float* kang = kang_all + (size_t)pr * kf_cap;
        int nm = 0, ne = 0;
        for (int i = 0; i < nk; ++i) {
            unsigned b = (unsigned)s.best[i];
            if (b == 0xFFFFFFFFu) continue;
            if (s.blocked[b & 0xFFFFu] != s.pre[b & 0xFFFFu])  // its best was taken meanwhile: re-scan
                b = reloc_scan(p, s, s.blocked, i, x3dc, dist, lvl, mpdesc, cdesc);
            if (b == 0xFFFFFFFFu || (int)(b >> 16) > p.orb_dist) continue;
            const int i2 = (int)(b & 0xFFFFu);
            s.assign[i2] = i;
            s.blocked[i2] = 1;
            ++nm;
            if (p.check_orientation) {
                float rot = kang[i] - K[i2].angle;
                if (rot < 0.0f) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == kProjHisto) bin = 0;
                s.ent[kf_cap + ne] = (unsigned short)bin;
                s.ent[ne++] = (unsigned short)i2;
                s_hist[bin]++;
            }
        }
        s_ne = ne;
        s_nm = nm;
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;  // ComputeThreeMaxima (:2304-2345)
        for (int b = 0; b < kProjHisto; b++) {
            const int c = s_hist[b];
            if (c > max1) {
                max3 = max2; max2 = max1; max1 = c;
                ind3 = ind2; ind2 = ind1; ind1 = b;
            } else if (c > max2) {
                max3 = max2; max2 = c;
                ind3 = ind2; ind2 = b;
            } else if (c > max3) {
                max3 = c;
                ind3 = b;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        s_keep[0] = ind1; s_keep[1] = ind2; s_keep[2] = ind3;
    }
    __syncthreads();
    // phase 3: entries in dropped bins set mvpMapPoints[idx] = NULL (:2284-2296)
    if (p.check_orientation) {
        const int ne = s_ne;
        int dropped = 0;
        for (int e = tid; e < ne; e += 256) {
            const int bin = s.ent[kf_cap + e];
            if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2]) {
                s.nulled[s.ent[e]] = 1;
                ++dropped;
            }
        }
        if (dropped) atomicSub(&s_nm, dropped);
        __syncthreads();
    }
    int* M = match + (size_t)pr * cur_cap;
    for (int i = tid; i < nc; i += 256) M[i] = s.nulled[i] ? -2 : s.assign[i];
    if (tid == 0) nmatches[pr] = s_nm;
}

static size_t local_smem(int cur_cap, int mp_cap) {
    return (size_t)cur_cap * (4 + 4 + 4 + 2 + 1 + 1 + 1) + (size_t)mp_cap * 8 + 4 * (kGridCells + 1) + 64;
}

static size_t local2_smem(int l_cap, int r_cap, int mp_cap) {
    auto side = [](int cap) { return ((size_t)cap * (4 + 4 + 4 + 2 + 1 + 1 + 1) + 4 * (kGridCells + 1) + 15) & ~size_t(15); };
    return 16 * (size_t)mp_cap + side(l_cap) + side(r_cap) + 64;
}

static size_t proj2_smem(int l_cap, int r_cap, int last_cap) {
    auto side = [](int cap) {
        return ((size_t)cap * (4 + 4 + 4 + 2 + 1 + 1 + 1 + 1) + 4 * (kGridCells + 1) + 15) & ~size_t(15);
    };
    return 16 * (size_t)last_cap + side(l_cap) + side(r_cap) + 64;
}

static size_t proj_smem(int cur_cap, int last_cap) {
    return (size_t)cur_cap * (4 + 4 + 4 + 2 + 1 + 1 + 1 + 1) + (size_t)last_cap * (4 + 4) + 4 * (kGridCells + 1) + 64;
}

static int grid_pow2(int cap) {
    int P = 256;
    while (P < cap) P <<= 1;
    return P;
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_assign_grid_batch(const plvi_keypoint* d_kps, const int* d_count, int cap, int n_frames,
                                      const plvi_grid_params* gp, int* d_cell_off, int* d_cell_idx, void* stream) {
    if (!gp || cap < 1 || cap > (1 << kGridKeyBits) || n_frames < 0) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    const int P = grid_pow2(cap);
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)assign_grid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  4 << kGridKeyBits);
    });
    hipLaunchKernelGGL(assign_grid_kernel, dim3(n_frames), dim3(256), (size_t)4 * P, (hipStream_t)stream, d_kps,
                       d_count, cap, P, *gp, d_cell_off, d_cell_idx);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_search_by_projection_batch(int n_pairs, const plvi_proj_params* p, const plvi_keypoint* d_cur_kps,
                                               const uint8_t* d_cur_desc, const int* d_cur_n, int cur_cap,
                                               const uint8_t* d_cur_blocked, const float* d_cur_uright,
                                               const int* d_cell_off, const int* d_cell_idx, const float* d_x3dc,
                                               const int* d_last_octave, const float* d_last_angle,
                                               const uint8_t* d_mp_desc, const uint8_t* d_last_flags,
                                               const int* d_last_n, int last_cap, int* d_match, int* d_nmatches,
                                               void* stream) {
    if (!p || n_pairs < 0 || cur_cap < 1 || last_cap < 1 || cur_cap > 65535 || last_cap > 65535) return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    const size_t smem = proj_smem(cur_cap, last_cap);
    if (!lds_fits<search_by_projection_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_by_projection_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    hipLaunchKernelGGL(search_by_projection_kernel, dim3(n_pairs), dim3(256), smem, (hipStream_t)stream, *p, d_cur_kps,
                       d_cur_desc, d_cur_n, cur_cap, d_cur_blocked, d_cur_uright, d_cell_off, d_cell_idx, d_x3dc,
                       d_last_octave, d_last_angle, d_mp_desc, d_last_flags, d_last_n, last_cap, d_match, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// One pair from host memory, synchronous (grid built on the device too).
// Returns nmatches (>= 0) or an error.
extern "C" int plvi_search_by_projection(const plvi_proj_params* p, const plvi_keypoint* cur_kps,
                                         const uint8_t* cur_desc, int n_cur, const uint8_t* cur_blocked,
                                         const float* cur_uright, const float* x3dc, const int* last_octave,
                                         const float* last_angle, const uint8_t* mp_desc, const uint8_t* last_flags,
                                         int n_last, int* match) {
    if (!p || n_cur < 0 || n_last < 0 || (n_cur > 0 && (!cur_kps || !cur_desc || !match))) return PLVI_E_BADARG;
    if (n_cur == 0) return 0;
    const int cc = n_cur, lc = std::max(n_last, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oK = put(sizeof(plvi_keypoint) * cc), oD = put(32 * (size_t)cc), oB = put(cc), oU = put(4 * (size_t)cc);
    const size_t oCO = put(4 * (size_t)(kGridCells + 1)), oCI = put(4 * (size_t)cc), oX = put(12 * (size_t)lc);
    const size_t oLO = put(4 * (size_t)lc), oLA = put(4 * (size_t)lc), oMD = put(32 * (size_t)lc), oLF = put(lc);
    const size_t oM = put(4 * (size_t)cc), oN = put(16);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oK, cur_kps, sizeof(plvi_keypoint) * cc) | up(oD, cur_desc, 32 * (size_t)cc);
    if (cur_blocked) rc |= up(oB, cur_blocked, cc);
    else PLVI_CHECK(hipMemset(B + off[oB], 0, cc));
    if (cur_uright) rc |= up(oU, cur_uright, 4 * (size_t)cc);
    if (n_last > 0)
        rc |= up(oX, x3dc, 12 * (size_t)n_last) | up(oLO, last_octave, 4 * (size_t)n_last) |
              up(oLA, last_angle, 4 * (size_t)n_last) | up(oMD, mp_desc, 32 * (size_t)n_last) |
              up(oLF, last_flags, n_last);
    if (rc) return PLVI_E_HIP;
    int counts[2] = {n_cur, n_last};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 8, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    plvi_grid_params gp{p->min_x, p->min_y, p->inv_w, p->inv_h};
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[oK]), dN, cc, 1, &gp,
                                reinterpret_cast<int*>(B + off[oCO]), reinterpret_cast<int*>(B + off[oCI]), nullptr);
    if (rc) return rc;
    rc = plvi_search_by_projection_batch(
        1, p, reinterpret_cast<const plvi_keypoint*>(B + off[oK]), B + off[oD], dN, cc, B + off[oB],
        cur_uright ? reinterpret_cast<const float*>(B + off[oU]) : nullptr, reinterpret_cast<const int*>(B + off[oCO]),
        reinterpret_cast<const int*>(B + off[oCI]), reinterpret_cast<const float*>(B + off[oX]),
        reinterpret_cast<const int*>(B + off[oLO]), reinterpret_cast<const float*>(B + off[oLA]), B + off[oMD],
        B + off[oLF], dN + 1, lc, reinterpret_cast<int*>(B + off[oM]), dN + 2, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nm = 0;
    PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n_cur, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nm, dN + 2, 4, hipMemcpyDeviceToHost));
    return nm;
}

extern "C" int plvi_search_reloc_batch(int n_pairs, const plvi_reloc_params* p, const plvi_keypoint* d_cur_kps,
                                       const uint8_t* d_cur_desc, const int* d_cur_n, int cur_cap,
                                       const uint8_t* d_cur_blocked, const int* d_cell_off, const int* d_cell_idx,
                                       const uint8_t* d_kf_flags, const float* d_x3dc, const float* d_dist,
                                       const int* d_level, const float* d_kf_angle, const uint8_t* d_mp_desc,
                                       const int* d_kf_n, int kf_cap, int* d_match, int* d_nmatches, void* stream) {
    if (!p || n_pairs < 0 || cur_cap < 1 || kf_cap < 1 || cur_cap > 65535 || kf_cap > 65535) return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16 || p->orb_dist < 0 || p->orb_dist > 255) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    const size_t smem = proj_smem(cur_cap, kf_cap);  // same carve-up as the frame-to-frame matcher
    if (!lds_fits<search_reloc_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_reloc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    hipLaunchKernelGGL(search_reloc_kernel, dim3(n_pairs), dim3(256), smem, (hipStream_t)stream, *p, d_cur_kps,
                       d_cur_desc, d_cur_n, cur_cap, d_cur_blocked, d_cell_off, d_cell_idx, d_kf_flags, d_x3dc, d_dist,
                       d_level, d_kf_angle, d_mp_desc, d_kf_n, kf_cap, d_match, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// One pair from host memory, synchronous (grid built on the device).
extern "C" int plvi_search_reloc(const plvi_reloc_params* p, const plvi_keypoint* cur_kps, const uint8_t* cur_desc,
                                 int n_cur, const uint8_t* cur_blocked, const uint8_t* kf_flags, const float* x3dc,
                                 const float* dist, const int* level, const float* kf_angle, const uint8_t* mp_desc,
                                 int n_kf, int* match) {
    if (!p || n_cur < 0 || n_kf < 0 || (n_cur > 0 && (!cur_kps || !cur_desc || !match))) return PLVI_E_BADARG;
    if (n_kf > 0 && (!kf_flags || !x3dc || !dist || !level || !kf_angle || !mp_desc)) return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16 || p->orb_dist < 0 || p->orb_dist > 255) return PLVI_E_BADARG;
    if (n_cur == 0) return 0;
    const int cc = n_cur, kc = std::max(n_kf, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oK = put(sizeof(plvi_keypoint) * cc), oD = put(32 * (size_t)cc), oB = put(cc);
    const size_t oCO = put(4 * (size_t)(kGridCells + 1)), oCI = put(4 * (size_t)cc), oF = put(kc);
    const size_t oX = put(12 * (size_t)kc), oS = put(12 * (size_t)kc), oL = put(4 * (size_t)kc);
    const size_t oA = put(4 * (size_t)kc), oMD = put(32 * (size_t)kc), oM = put(4 * (size_t)cc), oN = put(16);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oK, cur_kps, sizeof(plvi_keypoint) * cc) | up(oD, cur_desc, 32 * (size_t)cc);
    if (cur_blocked) rc |= up(oB, cur_blocked, cc);
    else PLVI_CHECK(hipMemset(B + off[oB], 0, cc));
    if (n_kf > 0)
        rc |= up(oF, kf_flags, n_kf) | up(oX, x3dc, 12 * (size_t)n_kf) | up(oS, dist, 12 * (size_t)n_kf) |
              up(oL, level, 4 * (size_t)n_kf) | up(oA, kf_angle, 4 * (size_t)n_kf) |
              up(oMD, mp_desc, 32 * (size_t)n_kf);
    if (rc) return PLVI_E_HIP;
    int counts[2] = {n_cur, n_kf};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 8, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    plvi_grid_params gp{p->min_x, p->min_y, p->inv_w, p->inv_h};
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[oK]), dN, cc, 1, &gp,
                                reinterpret_cast<int*>(B + off[oCO]), reinterpret_cast<int*>(B + off[oCI]), nullptr);
    if (rc) return rc;
    rc = plvi_search_reloc_batch(1, p, reinterpret_cast<const plvi_keypoint*>(B + off[oK]), B + off[oD], dN, cc,
                                 B + off[oB], reinterpret_cast<const int*>(B + off[oCO]),
                                 reinterpret_cast<const int*>(B + off[oCI]), B + off[oF],
                                 reinterpret_cast<const float*>(B + off[oX]), reinterpret_cast<const float*>(B + off[oS]),
                                 reinterpret_cast<const int*>(B + off[oL]), reinterpret_cast<const float*>(B + off[oA]),
                                 B + off[oMD], dN + 1, kc, reinterpret_cast<int*>(B + off[oM]), dN + 2, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nm = 0;
    PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n_cur, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nm, dN + 2, 4, hipMemcpyDeviceToHost));
    return nm;
}

extern "C" int plvi_search_local_batch(int n_frames, const plvi_local_params* p, const plvi_keypoint* d_kps,
                                       const uint8_t* d_desc, const int* d_n, int cap, const uint8_t* d_blocked,
                                       const float* d_uright, const int* d_cell_off, const int* d_cell_idx,
                                       const uint8_t* d_mp_flags, const float* d_mp_proj, const int* d_mp_level,
                                       const uint8_t* d_mp_desc, const int* d_mp_n, int mp_cap, int* d_match,
                                       int* d_nmatches, void* stream) {
    if (!p || n_frames < 0 || cap < 1 || mp_cap < 1 || cap > 65535) return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    const size_t smem = local_smem(cap, mp_cap);
    if (!lds_fits<search_local_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_local_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    hipLaunchKernelGGL(search_local_kernel, dim3(n_frames), dim3(256), smem, (hipStream_t)stream, *p, d_kps, d_desc,
                       d_n, cap, d_blocked, d_uright, d_cell_off, d_cell_idx, d_mp_flags, d_mp_proj, d_mp_level,
                       d_mp_desc, d_mp_n, mp_cap, d_match, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// One frame from host memory, synchronous (grid built on the device).
extern "C" int plvi_search_local(const plvi_local_params* p, const plvi_keypoint* kps, const uint8_t* desc, int n,
                                 const uint8_t* blocked, const float* uright, const uint8_t* mp_flags,
                                 const float* mp_proj, const int* mp_level, const uint8_t* mp_desc, int n_mp,
                                 int* match) {
    if (!p || n < 0 || n_mp < 0 || (n > 0 && (!kps || !desc || !match))) return PLVI_E_BADARG;
    if (n == 0) return 0;
    const int cc = n, mc = std::max(n_mp, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oK = put(sizeof(plvi_keypoint) * cc), oD = put(32 * (size_t)cc), oB = put(cc), oU = put(4 * (size_t)cc);
    const size_t oCO = put(4 * (size_t)(kGridCells + 1)), oCI = put(4 * (size_t)cc), oF = put(mc);
    const size_t oP = put(16 * (size_t)mc), oL = put(4 * (size_t)mc), oMD = put(32 * (size_t)mc);
    const size_t oM = put(4 * (size_t)cc), oN = put(16);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oK, kps, sizeof(plvi_keypoint) * cc) | up(oD, desc, 32 * (size_t)cc);
    if (blocked) rc |= up(oB, blocked, cc);
    else PLVI_CHECK(hipMemset(B + off[oB], 0, cc));
    if (uright) rc |= up(oU, uright, 4 * (size_t)cc);
    if (n_mp > 0)
        rc |= up(oF, mp_flags, n_mp) | up(oP, mp_proj, 16 * (size_t)n_mp) | up(oL, mp_level, 4 * (size_t)n_mp) |
              up(oMD, mp_desc, 32 * (size_t)n_mp);
    if (rc) return PLVI_E_HIP;
    int counts[2] = {n, n_mp};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 8, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    plvi_grid_params gp{p->min_x, p->min_y, p->inv_w, p->inv_h};
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[oK]), dN, cc, 1, &gp,
                                reinterpret_cast<int*>(B + off[oCO]), reinterpret_cast<int*>(B + off[oCI]), nullptr);
    if (rc) return rc;
    rc = plvi_search_local_batch(1, p, reinterpret_cast<const plvi_keypoint*>(B + off[oK]), B + off[oD], dN, cc,
                                 B + off[oB], uright ? reinterpret_cast<const float*>(B + off[oU]) : nullptr,
                                 reinterpret_cast<const int*>(B + off[oCO]), reinterpret_cast<const int*>(B + off[oCI]),
                                 B + off[oF], reinterpret_cast<const float*>(B + off[oP]),
                                 reinterpret_cast<const int*>(B + off[oL]), B + off[oMD], dN + 1, mc,
                                 reinterpret_cast<int*>(B + off[oM]), dN + 2, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nmt = 0;
    PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nmt, dN + 2, 4, hipMemcpyDeviceToHost));
    return nmt;
}

extern "C" int plvi_search_local_stereo_batch(
    int n_frames, const plvi_local_params* p, const plvi_keypoint* d_kps, const uint8_t* d_desc, const int* d_n,
    int cap, const uint8_t* d_blocked, const int* d_l2r, const int* d_cell_off, const int* d_cell_idx,
    const plvi_keypoint* d_kps_r, const uint8_t* d_desc_r, const int* d_n_r, int cap_r, const uint8_t* d_blocked_r,
    const int* d_r2l, const int* d_cell_off_r, const int* d_cell_idx_r, const uint8_t* d_mp_flags,
    const float* d_mp_proj, const int* d_mp_level, const float* d_mp_proj_r, const int* d_mp_level_r,
    const uint8_t* d_mp_desc, const int* d_mp_n, int mp_cap, int* d_match, int* d_match_r, int* d_nmatches,
    void* stream) {
    if (!p || n_frames < 0 || cap < 1 || cap_r < 1 || mp_cap < 1 || cap > 65535 || cap_r > 65535)
        return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    const size_t smem = local2_smem(cap, cap_r, mp_cap);
    if (!lds_fits<search_local2_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_local2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    hipLaunchKernelGGL(search_local2_kernel, dim3(n_frames), dim3(256), smem, (hipStream_t)stream, *p, d_kps, d_desc,
                       d_n, cap, d_blocked, d_l2r, d_cell_off, d_cell_idx, d_kps_r, d_desc_r, d_n_r, cap_r,
                       d_blocked_r, d_r2l, d_cell_off_r, d_cell_idx_r, d_mp_flags, d_mp_proj, d_mp_level, d_mp_proj_r,
                       d_mp_level_r, d_mp_desc, d_mp_n, mp_cap, d_match, d_match_r, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// One two-camera frame from host memory, synchronous (both grids built on the device).
extern "C" int plvi_search_local_stereo(const plvi_local_params* p, const plvi_keypoint* kps, const uint8_t* desc,
                                        int n, const uint8_t* blocked, const int* l2r, const plvi_keypoint* kps_r,
                                        const uint8_t* desc_r, int n_r, const uint8_t* blocked_r, const int* r2l,
                                        const uint8_t* mp_flags, const float* mp_proj, const int* mp_level,
                                        const float* mp_proj_r, const int* mp_level_r, const uint8_t* mp_desc,
                                        int n_mp, int* match, int* match_r) {
    if (!p || n < 0 || n_r < 0 || n_mp < 0) return PLVI_E_BADARG;
    if ((n > 0 && (!kps || !desc || !match)) || (n_r > 0 && (!kps_r || !desc_r || !match_r))) return PLVI_E_BADARG;
    if (n_mp > 0 && (!mp_flags || !mp_proj || !mp_level || !mp_proj_r || !mp_level_r || !mp_desc))
        return PLVI_E_BADARG;
    if (n + n_r == 0) return 0;
    const int cl = std::max(n, 1), cr = std::max(n_r, 1), mc = std::max(n_mp, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oK = put(sizeof(plvi_keypoint) * cl), oD = put(32 * (size_t)cl), oB = put(cl), oP2 = put(4 * (size_t)cl);
    const size_t oCO = put(4 * (size_t)(kGridCells + 1)), oCI = put(4 * (size_t)cl), oM = put(4 * (size_t)cl);
    const size_t rK = put(sizeof(plvi_keypoint) * cr), rD = put(32 * (size_t)cr), rB = put(cr), rP2 = put(4 * (size_t)cr);
    const size_t rCO = put(4 * (size_t)(kGridCells + 1)), rCI = put(4 * (size_t)cr), rM = put(4 * (size_t)cr);
    const size_t oF = put(mc), oP = put(16 * (size_t)mc), oL = put(4 * (size_t)mc), oPR = put(16 * (size_t)mc),
                 oLR = put(4 * (size_t)mc), oMD = put(32 * (size_t)mc), oN = put(16);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    PLVI_CHECK(hipMemset(B, 0, tot));
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oK, kps, sizeof(plvi_keypoint) * n) | up(oD, desc, 32 * (size_t)n) | up(oB, blocked, n) |
             up(rK, kps_r, sizeof(plvi_keypoint) * n_r) | up(rD, desc_r, 32 * (size_t)n_r) | up(rB, blocked_r, n_r);
    // no stereo pairs = every entry -1
    std::vector<int> none(std::max(n, n_r), -1);
    rc |= up(oP2, l2r ? l2r : none.data(), 4 * (size_t)n) | up(rP2, r2l ? r2l : none.data(), 4 * (size_t)n_r);
    if (n_mp > 0)
        rc |= up(oF, mp_flags, n_mp) | up(oP, mp_proj, 16 * (size_t)n_mp) | up(oL, mp_level, 4 * (size_t)n_mp) |
              up(oPR, mp_proj_r, 16 * (size_t)n_mp) | up(oLR, mp_level_r, 4 * (size_t)n_mp) |
              up(oMD, mp_desc, 32 * (size_t)n_mp);
    if (rc) return PLVI_E_HIP;
    int counts[4] = {n, n_r, n_mp, 0};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 16, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    plvi_grid_params gp{p->min_x, p->min_y, p->inv_w, p->inv_h};
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[oK]), dN, cl, 1, &gp,
                                reinterpret_cast<int*>(B + off[oCO]), reinterpret_cast<int*>(B + off[oCI]), nullptr);
    if (rc) return rc;
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[rK]), dN + 1, cr, 1, &gp,
                                reinterpret_cast<int*>(B + off[rCO]), reinterpret_cast<int*>(B + off[rCI]), nullptr);
    if (rc) return rc;
    rc = plvi_search_local_stereo_batch(
        1, p, reinterpret_cast<const plvi_keypoint*>(B + off[oK]), B + off[oD], dN, cl, B + off[oB],
        reinterpret_cast<const int*>(B + off[oP2]), reinterpret_cast<const int*>(B + off[oCO]),
        reinterpret_cast<const int*>(B + off[oCI]), reinterpret_cast<const plvi_keypoint*>(B + off[rK]), B + off[rD],
        dN + 1, cr, B + off[rB], reinterpret_cast<const int*>(B + off[rP2]), reinterpret_cast<const int*>(B + off[rCO]),
        reinterpret_cast<const int*>(B + off[rCI]), B + off[oF], reinterpret_cast<const float*>(B + off[oP]),
        reinterpret_cast<const int*>(B + off[oL]), reinterpret_cast<const float*>(B + off[oPR]),
        reinterpret_cast<const int*>(B + off[oLR]), B + off[oMD], dN + 2, mc, reinterpret_cast<int*>(B + off[oM]),
        reinterpret_cast<int*>(B + off[rM]), dN + 3, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nmt = 0;
    if (n) PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n, hipMemcpyDeviceToHost));
    if (n_r) PLVI_CHECK(hipMemcpy(match_r, B + off[rM], 4 * (size_t)n_r, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nmt, dN + 3, 4, hipMemcpyDeviceToHost));
    return nmt;
}

extern "C" int plvi_search_by_projection_stereo_batch(
    int n_pairs, const plvi_proj_params* p, const float* kb8, const plvi_keypoint* d_kps, const uint8_t* d_desc,
    const int* d_n, int cap, const uint8_t* d_blocked, const int* d_cell_off, const int* d_cell_idx,
    const plvi_keypoint* d_kps_r, const uint8_t* d_desc_r, const int* d_n_r, int cap_r, const uint8_t* d_blocked_r,
    const int* d_cell_off_r, const int* d_cell_idx_r, const float* d_x3dc, const float* d_x3dr,
    const int* d_last_octave, const float* d_last_angle, const uint8_t* d_mp_desc, const uint8_t* d_last_flags,
    const int* d_last_n, int last_cap, int* d_match, int* d_match_r, int* d_nmatches, void* stream) {
    if (!p || n_pairs < 0 || cap < 1 || cap_r < 1 || last_cap < 1 || cap > 65535 || cap_r > 65535 ||
        last_cap > 65535)
        return PLVI_E_BADARG;
    if (p->nlevels < 1 || p->nlevels > 16) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    const size_t smem = proj2_smem(cap, cap_r, last_cap);
    if (!lds_fits<search_by_projection2_kernel>(smem)) return PLVI_E_CAPACITY;
    CamModel cm{0, 0.f, 0.f, 0.f, 0.f};
    if (kb8) cm = CamModel{1, kb8[0], kb8[1], kb8[2], kb8[3]};
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_by_projection2_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    hipLaunchKernelGGL(search_by_projection2_kernel, dim3(n_pairs), dim3(256), smem, (hipStream_t)stream, *p, cm, d_kps,
                       d_desc, d_n, cap, d_blocked, d_cell_off, d_cell_idx, d_kps_r, d_desc_r, d_n_r, cap_r,
                       d_blocked_r, d_cell_off_r, d_cell_idx_r, d_x3dc, d_x3dr, d_last_octave, d_last_angle, d_mp_desc,
                       d_last_flags, d_last_n, last_cap, d_match, d_match_r, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// One pair from host memory, synchronous (both grids built on the device).
extern "C" int plvi_search_by_projection_stereo(const plvi_proj_params* p, const float* kb8, const plvi_keypoint* kps,
                                                const uint8_t* desc, int n, const uint8_t* blocked,
                                                const plvi_keypoint* kps_r, const uint8_t* desc_r, int n_r,
                                                const uint8_t* blocked_r, const float* x3dc, const float* x3dr,
                                                const int* last_octave, const float* last_angle,
                                                const uint8_t* mp_desc, const uint8_t* last_flags, int n_last,
                                                int* match, int* match_r) {
    if (!p || n < 0 || n_r < 0 || n_last < 0) return PLVI_E_BADARG;
    if ((n > 0 && (!kps || !desc || !match)) || (n_r > 0 && (!kps_r || !desc_r || !match_r))) return PLVI_E_BADARG;
    if (n_last > 0 && (!x3dc || !x3dr || !last_octave || !last_angle || !mp_desc || !last_flags)) return PLVI_E_BADARG;
    const int cl = std::max(n, 1), cr = std::max(n_r, 1), lc = std::max(n_last, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oK = put(sizeof(plvi_keypoint) * cl), oD = put(32 * (size_t)cl), oB = put(cl);
    const size_t oCO = put(4 * (size_t)(kGridCells + 1)), oCI = put(4 * (size_t)cl), oM = put(4 * (size_t)cl);
    const size_t rK = put(sizeof(plvi_keypoint) * cr), rD = put(32 * (size_t)cr), rB = put(cr);
    const size_t rCO = put(4 * (size_t)(kGridCells + 1)), rCI = put(4 * (size_t)cr), rM = put(4 * (size_t)cr);
    const size_t oX = put(12 * (size_t)lc), oXR = put(12 * (size_t)lc), oO = put(4 * (size_t)lc),
                 oA = put(4 * (size_t)lc), oMD = put(32 * (size_t)lc), oF = put(lc), oN = put(16);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    PLVI_CHECK(hipMemset(B, 0, tot));
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oK, kps, sizeof(plvi_keypoint) * n) | up(oD, desc, 32 * (size_t)n) | up(oB, blocked, n) |
             up(rK, kps_r, sizeof(plvi_keypoint) * n_r) | up(rD, desc_r, 32 * (size_t)n_r) | up(rB, blocked_r, n_r) |
             up(oX, x3dc, 12 * (size_t)n_last) | up(oXR, x3dr, 12 * (size_t)n_last) |
             up(oO, last_octave, 4 * (size_t)n_last) | up(oA, last_angle, 4 * (size_t)n_last) |
             up(oMD, mp_desc, 32 * (size_t)n_last) | up(oF, last_flags, n_last);
    if (rc) return PLVI_E_HIP;
    int counts[4] = {n, n_r, n_last, 0};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 16, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    plvi_grid_params gp{p->min_x, p->min_y, p->inv_w, p->inv_h};
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[oK]), dN, cl, 1, &gp,
                                reinterpret_cast<int*>(B + off[oCO]), reinterpret_cast<int*>(B + off[oCI]), nullptr);
    if (rc) return rc;
    rc = plvi_assign_grid_batch(reinterpret_cast<const plvi_keypoint*>(B + off[rK]), dN + 1, cr, 1, &gp,
                                reinterpret_cast<int*>(B + off[rCO]), reinterpret_cast<int*>(B + off[rCI]), nullptr);
    if (rc) return rc;
    rc = plvi_search_by_projection_stereo_batch(
        1, p, kb8, reinterpret_cast<const plvi_keypoint*>(B + off[oK]), B + off[oD], dN, cl, B + off[oB],
        reinterpret_cast<const int*>(B + off[oCO]), reinterpret_cast<const int*>(B + off[oCI]),
        reinterpret_cast<const plvi_keypoint*>(B + off[rK]), B + off[rD], dN + 1, cr, B + off[rB],
        reinterpret_cast<const int*>(B + off[rCO]), reinterpret_cast<const int*>(B + off[rCI]),
        reinterpret_cast<const float*>(B + off[oX]), reinterpret_cast<const float*>(B + off[oXR]),
        reinterpret_cast<const int*>(B + off[oO]), reinterpret_cast<const float*>(B + off[oA]), B + off[oMD],
        B + off[oF], dN + 2, lc, reinterpret_cast<int*>(B + off[oM]), reinterpret_cast<int*>(B + off[rM]), dN + 3,
        nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int nmt = 0;
    if (n) PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n, hipMemcpyDeviceToHost));
    if (n_r) PLVI_CHECK(hipMemcpy(match_r, B + off[rM], 4 * (size_t)n_r, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nmt, dN + 3, 4, hipMemcpyDeviceToHost));
    return nmt;
}
