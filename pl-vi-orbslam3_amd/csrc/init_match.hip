// init_match.hip — the monocular initializer's matchers, run on every frame
// until Tracking::MonocularInitialization succeeds (src/Tracking.cc:3111-3113):
//   ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12,
//     windowSize)                       src/ORBmatcher.cc:705-814
//   LineMatcher::SerachForInitialize    src/LineMatcher.cpp:113-139
//     + Frame::lineDescriptorMAD        src/Frame.cc:1089-1112
//
// SearchForInitialization, one 4-wave workgroup per (F1, F2) pair.  The scan
// of F1 keypoint i1 depends on earlier keypoints only through
// vMatchedDistance (a candidate i2 is skipped while vMatchedDistance[i2] <=
// dist), which only decreases.  Phase 1: every level-0 keypoint's window is
// scanned with no candidate excluded, a wave per keypoint (lanes over the
// window's grid cells, 64-bit keys dist | scan position | index give the
// reference's first-achiever argmin and the second-smallest distance).
// Phase 2, one wave in F1 order: a keypoint whose best or second candidate
// is now excluded is re-scanned against the current vMatchedDistance
// (excluding any other candidate changes neither); then the ratio test, the
// steal of a previously matched i2 and the rotation histogram as in the
// reference.  Phase 3: ComputeThreeMaxima and the filter, then vbPrevMatched.
//
// SerachForInitialize: knnMatch(k = 2) by hamming_knn2_kernel (match.hip),
// then one workgroup per pair computes lineDescriptorMAD's medians as order
// statistics of integer keys (distances <= 256: LDS histograms instead of
// the reference's std::sort of the match lists -- the element at index n/2
// of a sorted list is the n/2-th order statistic whatever the sort) and
// emits the pairs with d1 - d0 > 0.5 * nn12_mad in query order.
#include <hip/hip_runtime.h>

#include <climits>
#include <vector>

#include "plvi_common.h"

namespace plvi {

int launch_knn2(const uint8_t* q, const int* nq, int nq_cap, const uint8_t* t, const int* nt, int nt_cap,
                int n_pairs, int* i0, int* d0, int* i1, int* d1, hipStream_t st);

namespace {
constexpr int kCols = 64, kRows = 48, kCells = kCols * kRows;  // FRAME_GRID_COLS / ROWS (include/Frame.h:47-48)
constexpr int kThLow = 50, kHisto = 30;                        // ORBmatcher::TH_LOW, HISTO_LENGTH
constexpr unsigned long long kNoKey = ~0ull;

struct InitLds {
    float *kx, *ky;
    int *cell_off, *md, *v21, *v12;
    unsigned long long *best, *sec;
    unsigned short *cell_idx, *ent;
    unsigned char* k0;  // F2 keypoint has octave 0
};

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
        const unsigned long long o = __shfl_xor(v, s);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int dist256(const uint4 a0, const uint4 a1, const uint8_t* __restrict__ b) {
    const uint4* pb = reinterpret_cast<const uint4*>(b);
    const uint4 b0 = pb[0], b1 = pb[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// GetFeaturesInArea(x, y, r, 0, 0) (Frame.cc:1006-1075) + the candidate loop
// of SearchForInitialization (:728-753) over the window, one wave: returns
// best key in `best` (dist << 40 | scan position << 16 | i2) and the key of a
// candidate holding the second-smallest distance in `sec` (kNoKey: none).
// md == nullptr: no candidate excluded (vMatchedDistance all INT_MAX).
__device__ void init_scan(const plvi_init_params& p, const InitLds& s, const int* md, float x, float y, uint4 a0,
                          uint4 a1, const uint8_t* __restrict__ desc2, int lane, unsigned long long& best,
                          unsigned long long& sec) {
    best = sec = kNoKey;
    const float r = (float)p.window;
    const int nMinCellX = max(0, (int)floorf((x - p.min_x - r) * p.inv_w));
    if (nMinCellX >= kCols) return;
    const int nMaxCellX = min(kCols - 1, (int)ceilf((x - p.min_x + r) * p.inv_w));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - p.min_y - r) * p.inv_h));
    if (nMinCellY >= kRows) return;
    const int nMaxCellY = min(kRows - 1, (int)ceilf((y - p.min_y + r) * p.inv_h));
    if (nMaxCellY < 0) return;
    unsigned long long k1 = kNoKey, k2 = kNoKey;
    int pos = 0;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        // cells (ix, nMinCellY..nMaxCellY) are one CSR range, in mGrid scan order
        const int c0 = s.cell_off[ix * kRows + nMinCellY], c1 = s.cell_off[ix * kRows + nMaxCellY + 1];
        for (int k = c0 + lane; k < c1; k += 64) {
            const int i2 = s.cell_idx[k];
            if (!s.k0[i2]) continue;  // octave < 0 or > 0
            const float distx = s.kx[i2] - x, disty = s.ky[i2] - y;
            if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
            const int dist = dist256(a0, a1, desc2 + (size_t)32 * i2);
            if (md && md[i2] <= dist) continue;
            const unsigned long long key =
                ((unsigned long long)dist << 40) | ((unsigned long long)(pos + k - c0) << 16) | (unsigned)i2;
            if (key < k1) {
                k2 = k1;
                k1 = key;
            } else if (key < k2) {
                k2 = key;
            }
        }
        pos += c1 - c0;
    }
    best = wave_min_u64(k1);
    sec = wave_min_u64(k1 == best ? k2 : k1);
}
}  // namespace

__global__ __launch_bounds__(256) void search_init_kernel(
    plvi_init_params p, const plvi_keypoint* __restrict__ kps1_all, const uint8_t* __restrict__ desc1_all,
    const int* __restrict__ n1_all, int cap1, float* __restrict__ prev_all, const plvi_keypoint* __restrict__ kps2_all,
    const uint8_t* __restrict__ desc2_all, const int* __restrict__ n2_all, int cap2, const int* __restrict__ cell_off_all,
    const int* __restrict__ cell_idx_all, int* __restrict__ m12_all, int* __restrict__ nmatch_all) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int pr = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n1 = min(n1_all[pr], cap1), n2 = min(n2_all[pr], cap2);
    InitLds s;
    {
        unsigned char* q = lds;
        s.best = reinterpret_cast<unsigned long long*>(q); q += 8 * (size_t)cap1;
        s.sec = reinterpret_cast<unsigned long long*>(q); q += 8 * (size_t)cap1;
        s.kx = reinterpret_cast<float*>(q); q += 4 * (size_t)cap2;
        s.ky = reinterpret_cast<float*>(q); q += 4 * (size_t)cap2;
        s.md = reinterpret_cast<int*>(q); q += 4 * (size_t)cap2;
        s.v21 = reinterpret_cast<int*>(q); q += 4 * (size_t)cap2;
        s.v12 = reinterpret_cast<int*>(q); q += 4 * (size_t)cap1;
        s.cell_off = reinterpret_cast<int*>(q); q += 4 * (kCells + 1);
        s.cell_idx = reinterpret_cast<unsigned short*>(q); q += 2 * (size_t)cap2;
        s.ent = reinterpret_cast<unsigned short*>(q); q += 4 * (size_t)cap1;  // [cap1] i1, [cap1] bin
        s.k0 = q;
    }
    __shared__ int s_hist[kHisto], s_keep[3], s_ne, s_nm;
    const plvi_keypoint* K1 = kps1_all + (size_t)pr * cap1;
    const plvi_keypoint* K2 = kps2_all + (size_t)pr * cap2;
    const uint8_t* D1 = desc1_all + (size_t)pr * cap1 * 32;
    const uint8_t* D2 = desc2_all + (size_t)pr * cap2 * 32;
    float* prev = prev_all + (size_t)pr * cap1 * 2;
    for (int i = tid; i < n2; i += 256) {
        s.kx[i] = K2[i].x;
        s.ky[i] = K2[i].y;
        s.k0[i] = K2[i].octave == 0;
        s.md[i] = INT_MAX;
        s.v21[i] = -1;
    }
    for (int i = tid; i < n1; i += 256) s.v12[i] = -1;
    const int* CO = cell_off_all + (size_t)pr * (kCells + 1);
    for (int c = tid; c <= kCells; c += 256) s.cell_off[c] = CO[c];
    const int ncell = CO[kCells];
    for (int k = tid; k < ncell; k += 256) s.cell_idx[k] = (unsigned short)cell_idx_all[(size_t)pr * cap2 + k];
    if (tid < kHisto) s_hist[tid] = 0;
    __syncthreads();
    // phase 1: every level-0 keypoint against all its candidates, a wave each
    for (int i1 = wv; i1 < n1; i1 += 4) {
        if (K1[i1].octave > 0) continue;  // level1 > 0 (:722-724)
        const uint4* pa = reinterpret_cast<const uint4*>(D1 + (size_t)32 * i1);
        unsigned long long b, c;
        init_scan(p, s, nullptr, prev[2 * i1], prev[2 * i1 + 1], pa[0], pa[1], D2, lane, b, c);
        if (lane == 0) {
            s.best[i1] = b;
            s.sec[i1] = c;
        }
    }
    __syncthreads();
    // phase 2: the assignment in F1 order (:755-781), one wave
    if (wv == 0) {
        const float factor = 1.0f / kHisto;
        int nm = 0, ne = 0;
        for (int i1 = 0; i1 < n1; ++i1) {
            if (K1[i1].octave > 0) continue;
            unsigned long long b = s.best[i1], c = s.sec[i1];
            if (b == kNoKey) continue;  // empty window or no candidate
            const int bi = (int)(b & 0xffffu), bd = (int)(b >> 40);
            const bool stale = s.md[bi] <= bd || (c != kNoKey && s.md[(int)(c & 0xffffu)] <= (int)(c >> 40));
            if (stale) {
                const uint4* pa = reinterpret_cast<const uint4*>(D1 + (size_t)32 * i1);
                init_scan(p, s, s.md, prev[2 * i1], prev[2 * i1 + 1], pa[0], pa[1], D2, lane, b, c);
                if (b == kNoKey) continue;
            }
            const int bestDist = (int)(b >> 40), bestIdx2 = (int)(b & 0xffffu);
            const int bestDist2 = c == kNoKey ? INT_MAX : (int)(c >> 40);
            if (bestDist <= kThLow && (float)bestDist < (float)bestDist2 * p.nnratio) {
                if (lane == 0) {
                    const int prev1 = s.v21[bestIdx2];
                    if (prev1 >= 0) s.v12[prev1] = -1;
                    s.v12[i1] = bestIdx2;
                    s.v21[bestIdx2] = i1;
                    s.md[bestIdx2] = bestDist;
                    if (p.check_orientation) {
                        float rot = K1[i1].angle - K2[bestIdx2].angle;
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == kHisto) bin = 0;
                        s.ent[ne] = (unsigned short)i1;
                        s.ent[cap1 + ne] = (unsigned short)bin;
                        s_hist[bin]++;
                    }
                }
                if (p.check_orientation) ++ne;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (lane == 0) {
            // nmatches = live entries of vnMatches12 before the rotation filter
            // (every steal removed exactly one)
            for (int i1 = 0; i1 < n1; ++i1) nm += s.v12[i1] >= 0;
            s_ne = ne;
            s_nm = nm;
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;  // ComputeThreeMaxima (:2304-2345)
            for (int bb = 0; bb < kHisto; bb++) {
                const int cnt = s_hist[bb];
                if (cnt > max1) {
                    max3 = max2; max2 = max1; max1 = cnt;
                    ind3 = ind2; ind2 = ind1; ind1 = bb;
                } else if (cnt > max2) {
                    max3 = max2; max2 = cnt;
                    ind3 = ind2; ind2 = bb;
                } else if (cnt > max3) {
                    max3 = cnt;
                    ind3 = bb;
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
    }
    __syncthreads();
    // phase 3: the rotation filter (:784-805); an F1 keypoint appears once
    if (p.check_orientation) {
        int dropped = 0;
        for (int e = tid; e < s_ne; e += 256) {
            const int bin = s.ent[cap1 + e], i1 = s.ent[e];
            if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2] && s.v12[i1] >= 0) {
                s.v12[i1] = -1;
                ++dropped;
            }
        }
        if (dropped) atomicSub(&s_nm, dropped);
        __syncthreads();
    }
    // vnMatches12 and the updated vbPrevMatched (:808-811)
    int* M = m12_all + (size_t)pr * cap1;
    for (int i1 = tid; i1 < n1; i1 += 256) {
        const int m = s.v12[i1];
        M[i1] = m;
        if (m >= 0) {
            prev[2 * i1] = K2[m].x;
            prev[2 * i1 + 1] = K2[m].y;
        }
    }
    if (tid == 0) nmatch_all[pr] = s_nm;
}

// lineDescriptorMAD + the selection of SerachForInitialize, one workgroup per
// pair, from the kNN-2 tables (i0, d0, i1, d1) [pair][cap1].
__global__ __launch_bounds__(256) void line_init_select_kernel(const int* __restrict__ n1_all, int cap1,
                                                               const int* __restrict__ n2_all,
                                                               const int* __restrict__ i0_all,
                                                               const int* __restrict__ d0_all,
                                                               const int* __restrict__ d1_all, int2* __restrict__ out,
                                                               int* __restrict__ nout, double* __restrict__ mad) {
    __shared__ int h[4][260];
    __shared__ int s_med[2], s_dev[2], s_wsum[4];
    const int pr = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n1 = min(n1_all[pr], cap1), n2 = n2_all[pr];
    if (n1 <= 0 || n2 < 2) {  // the reference reads lmatches[0] / [i][1]: undefined, no pairs here
        if (tid == 0) {
            nout[pr] = 0;
            if (mad) mad[2 * pr] = mad[2 * pr + 1] = 0.0;
        }
        return;
    }
    const int* D0 = d0_all + (size_t)pr * cap1;
    const int* D1 = d1_all + (size_t)pr * cap1;
    const int* I0 = i0_all + (size_t)pr * cap1;
    for (int k = tid; k < 4 * 260; k += 256) (&h[0][0])[k] = 0;
    __syncthreads();
    // histograms of the NN distance and of d1 - d0 (both in [0, 256])
    for (int i = tid; i < n1; i += 256) {
        atomicAdd(&h[0][D0[i]], 1);
        atomicAdd(&h[1][D1[i] - D0[i]], 1);
    }
    __syncthreads();
    // the k-th smallest of a histogram (k = n1 / 2; d1 - d0 is sorted
    // descending by conpare_descriptor_by_NN12_dist: its index n1/2 is the
    // (n1 - 1 - n1/2)-th smallest)
    if (tid < 2) {
        const int k = tid == 0 ? n1 / 2 : n1 - 1 - n1 / 2;
        int acc = 0, v = 0;
        for (; v <= 256; ++v) {
            acc += h[tid][v];
            if (acc > k) break;
        }
        s_med[tid] = v;
    }
    __syncthreads();
    for (int i = tid; i < n1; i += 256) {
        atomicAdd(&h[2][abs(D0[i] - s_med[0])], 1);
        atomicAdd(&h[3][abs(D1[i] - D0[i] - s_med[1])], 1);
    }
    __syncthreads();
    if (tid < 2) {
        const int k = n1 / 2;  // both deviation lists sorted ascending (compare_descriptor_by_NN_dist)
        int acc = 0, v = 0;
        for (; v <= 256; ++v) {
            acc += h[2 + tid][v];
            if (acc > k) break;
        }
        s_dev[tid] = v;
    }
    __syncthreads();
    const double nn_mad = 1.4826 * (double)(float)s_dev[0];
    const double nn12_mad = 1.4826 * (double)(float)s_dev[1];
    const double th = nn12_mad * 0.5;
    if (mad && tid == 0) {
        mad[2 * pr] = nn_mad;
        mad[2 * pr + 1] = nn12_mad;
    }
    // LineMatches in query order: (double)(d1 - d0) > 0.5 * nn12_mad
    int2* O = out + (size_t)pr * cap1;
    int base = 0;
    for (int i0 = 0; i0 < n1; i0 += 256) {
        const int i = i0 + tid;
        const bool keep = i < n1 && (double)((float)D1[i] - (float)D0[i]) > th;
        const unsigned long long b = __ballot(keep);
        if (lane == 0) s_wsum[wv] = __popcll(b);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wv; ++w) off += s_wsum[w];
        if (keep) O[off + __popcll(b & ((1ull << lane) - 1ull))] = make_int2(i, I0[i]);
        base += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
        __syncthreads();
    }
    if (tid == 0) nout[pr] = base;
}

static size_t init_smem(int cap1, int cap2) {
    return (size_t)cap1 * (8 + 8 + 4 + 4) + (size_t)cap2 * (4 + 4 + 4 + 4 + 2 + 1) + 4 * (kCells + 1) + 64;
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_search_for_initialization_batch(int n_pairs, const plvi_init_params* p,
                                                    const plvi_keypoint* d_kps1, const uint8_t* d_desc1,
                                                    const int* d_n1, int cap1, float* d_prev_matched,
                                                    const plvi_keypoint* d_kps2, const uint8_t* d_desc2,
                                                    const int* d_n2, int cap2, const int* d_cell_off,
                                                    const int* d_cell_idx, int* d_matches12, int* d_nmatches,
                                                    void* stream) {
    if (!p || n_pairs < 0 || cap1 < 1 || cap2 < 1 || cap1 > 65535 || cap2 > 65535) return PLVI_E_BADARG;
    if (!(p->window > 0)) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    const size_t smem = init_smem(cap1, cap2);
    // (with the kernel's static __shared__ histogram, kept bins, counters)
    if (!lds_fits<search_init_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)search_init_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    hipLaunchKernelGGL(search_init_kernel, dim3(n_pairs), dim3(256), smem, (hipStream_t)stream, *p, d_kps1, d_desc1,
                       d_n1, cap1, d_prev_matched, d_kps2, d_desc2, d_n2, cap2, d_cell_off, d_cell_idx, d_matches12,
                       d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_line_search_init_batch(const uint8_t* d_desc1, const int* d_n1, int cap1, const uint8_t* d_desc2,
                                           const int* d_n2, int cap2, int n_pairs, int* d_scratch, int* d_pairs,
                                           int* d_npairs, double* d_mad, void* stream) {
    if (n_pairs < 0 || cap1 < 1 || cap2 < 1) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    if (!d_desc1 || !d_n1 || !d_desc2 || !d_n2 || !d_scratch || !d_pairs || !d_npairs) return PLVI_E_BADARG;
    const size_t plane = (size_t)n_pairs * cap1;
    int* i0 = d_scratch;
    int* d0 = d_scratch + plane;
    int* i1 = d_scratch + 2 * plane;
    int* d1 = d_scratch + 3 * plane;
    const hipStream_t st = (hipStream_t)stream;
    if (int rc = launch_knn2(d_desc1, d_n1, cap1, d_desc2, d_n2, cap2, n_pairs, i0, d0, i1, d1, st)) return rc;
    hipLaunchKernelGGL(line_init_select_kernel, dim3(n_pairs), dim3(256), 0, st, d_n1, cap1, d_n2, i0, d0, d1,
                       reinterpret_cast<int2*>(d_pairs), d_npairs, d_mad);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}
