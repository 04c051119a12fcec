// proj.hip — the steady-state frame-to-frame ORB matcher on the device:
//   Frame::AssignFeaturesToGrid (src/Frame.cc:644-675) + PosInGrid (:1077-1087)
//   Frame::GetFeaturesInArea (src/Frame.cc:1006-1075)
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//     (src/ORBmatcher.cc:1962-2178, Nleft == -1 branch) + ComputeThreeMaxima
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
                const float ur = u - p.mbf * invzc;
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
    if (smem > 160 * 1024) return PLVI_E_CAPACITY;
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
