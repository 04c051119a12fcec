// stereo.hip — rectified stereo matching of the stereo Frame constructors
// (src/Frame.cc:95-140 ORB, :225-300 ORB + lines), batched over frame pairs:
//
//   Frame::ComputeStereoMatches        src/Frame.cc:1228-1406
//     stereo_orb_kernel: one workgroup per pair.  The right keypoints are
//     bucketed by row in LDS (vRowIndices, :1238-1255); one thread per left
//     keypoint takes the min of (Hamming, right index) over its row bucket,
//     which is the reference's strict-< first-wins scan in index order
//     (:1284-1311); the 11 x 11 SAD window search (:1323-1358) runs one wave
//     per surviving keypoint, lane = (offset, window row); the median
//     outlier rejection (:1392-1405) is a 16-bit radix select of the median
//     SAD followed by a parallel threshold test (rejects exactly the sorted
//     tail the reference walks).
//   Frame::ComputeStereoMatches_Lines  src/Frame.cc:1408-1492
//     stereo_line_grid_kernel: line_2d coordinates of the left lines, the
//     normalised right directions and the 64 x 48 GridStructure of the right
//     lines (getLineCoords = LineIterator, src/gridStructure.cpp:32-40,
//     src/LineIterator.cpp:31-73) as CSR with cells in push_back (= index)
//     order; then LineMatcher::matchGrid (grid_match.hip); then
//     stereo_line_disparity_kernel: endpoint disparities
//     (lineSegmentOverlapStereo :1494-1529, filterLineSegmentDisparity
//     :1531-1542, including the reference's reuse of the updated sp_r when
//     it re-projects ep_r, :1469-1470) and mvle_l (:1486-1491).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "plvi_common.h"
#include "plvi_math.h"

namespace plvi {

constexpr int kStThreads = 256;
constexpr int kThHigh = 100, kThLow = 50;          // ORBmatcher::TH_HIGH / TH_LOW
constexpr int kLGridCols = 64, kLGridRows = 48;    // FRAME_GRID_COLS / ROWS (include/Frame.h:47-48)
constexpr int kLGridCells = kLGridCols * kLGridRows;

// per level and side: frame 0's image and the bytes between frames (level 0
// may be a view of the caller's frames, the other levels the extractor's
// pyramid buffer: plvi_orb_pyramid_device)
struct StereoLv {
    const uint8_t* pl[16];
    const uint8_t* pr[16];
    long long planeL[16], planeR[16];
    int w[16], h[16];
};
struct StereoPrm {
    float mb, mbf;
    int nlevels, rowCap;
    float scale[16], inv[16];
};

__device__ __forceinline__ int hamming32(const uint4* a, const uint4* b) {
    const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Exclusive scan of s[0..n) in place over the 256-thread block; returns the total.
__device__ int block_scan_excl(int* s, int n, int* s_tmp) {
    const int t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int per = (n + kStThreads - 1) / kStThreads, b0 = min(n, t * per), b1 = min(n, b0 + per);
    int local = 0;
    for (int i = b0; i < b1; ++i) local += s[i];
    int x = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kStThreads / 64; ++w) {
        base += w < wv ? s_tmp[w] : 0;
        tot += s_tmp[w];
    }
    int run = base + x - local;
    for (int i = b0; i < b1; ++i) {
        const int v = s[i];
        s[i] = run;
        run += v;
    }
    __syncthreads();
    return tot;
}

// ---------------------------------------------------------------------------
// Frame::ComputeStereoMatches (src/Frame.cc:1228-1406)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kStThreads) void stereo_orb_kernel(
    const plvi_keypoint* __restrict__ kL, const uint8_t* __restrict__ dL, const int* __restrict__ nLs, int capL,
    const plvi_keypoint* __restrict__ kR, const uint8_t* __restrict__ dR, const int* __restrict__ nRs, int capR,
    StereoLv lv, StereoPrm prm, float* __restrict__ uright, float* __restrict__ depth, int* __restrict__ nstereo, int* __restrict__ err) {
    extern __shared__ __align__(16) int lds_s[];
    __shared__ int s_tmp[kStThreads / 64], s_njob, s_nacc, s_fail, s_hist[256], s_sel[2];
    __shared__ int s_part[kStThreads / 64][121], s_dist[kStThreads / 64][11];
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int nL = nLs[f], nR = nRs[f];
    const int nRows = lv.h[0];
    int* s_row = lds_s;                                        // nRows + 1 (counts -> offsets)
    int* s_cur = s_row + (nRows + 1);                          // nRows fill cursors
    float* s_rx = reinterpret_cast<float*>(s_cur + nRows);     // capR right u
    int* s_roct = reinterpret_cast<int*>(s_rx + capR);         // capR right octave
    int* s_res = s_roct + capR;                                // capL: best right index / accepted SAD
    int* s_job = s_res + capL;                                 // capL: SAD jobs
    float* s_ur = reinterpret_cast<float*>(s_job + capL);      // capL mvuRight
    float* s_dp = s_ur + capL;                                 // capL mvDepth
    unsigned short* s_idx = reinterpret_cast<unsigned short*>(s_dp + capL);  // rowCap bucket entries
    const plvi_keypoint* KL = kL + (size_t)f * capL;
    const plvi_keypoint* KR = kR + (size_t)f * capR;
    const uint8_t* DL = dL + (size_t)f * capL * 32;
    const uint8_t* DR = dR + (size_t)f * capR * 32;
    for (int i = t; i <= nRows; i += kStThreads) s_row[i] = 0;
    for (int i = t; i < nRows; i += kStThreads) s_cur[i] = 0;
    for (int i = t; i < nL; i += kStThreads) { s_ur[i] = -1.0f; s_dp[i] = -1.0f; s_res[i] = -1; }
    if (t == 0) { s_njob = 0; s_nacc = 0; s_fail = 0; }
    __syncthreads();
    // vRowIndices (:1238-1255)
    for (int iR = t; iR < nR; iR += kStThreads) {
        const plvi_keypoint kp = KR[iR];
        // ceil(kpY + r) / floor(kpY - r), r = 2*scale: fused in Frame.cc.o
        const int maxr = (int)__builtin_ceilf(rfmaf(2.0f, prm.scale[kp.octave], kp.y));
        const int minr = (int)__builtin_floorf(rfmaf(-2.0f, prm.scale[kp.octave], kp.y));
        s_rx[iR] = kp.x;
        s_roct[iR] = kp.octave;
        if (minr < 0 || maxr >= nRows) { s_fail = 1; continue; }  // vRowIndices[yi] out of range (UB)
        for (int yi = minr; yi <= maxr; ++yi) atomicAdd(&s_row[yi], 1);
    }
    __syncthreads();
    const int total = block_scan_excl(s_row, nRows + 1, s_tmp);
    if (total > prm.rowCap) s_fail = 1;
    __syncthreads();
    if (s_fail) {
        for (int i = t; i < nL; i += kStThreads) {
            uright[(size_t)f * capL + i] = -1.0f;
            depth[(size_t)f * capL + i] = -1.0f;
        }
        if (t == 0) { atomicOr(err, 1); nstereo[f] = 0; }
        return;
    }
    for (int iR = t; iR < nR; iR += kStThreads) {
        const float y = KR[iR].y, sc = prm.scale[s_roct[iR]];
        const int maxr = (int)__builtin_ceilf(rfmaf(2.0f, sc, y)), minr = (int)__builtin_floorf(rfmaf(-2.0f, sc, y));
        for (int yi = minr; yi <= maxr; ++yi) s_idx[s_row[yi] + atomicAdd(&s_cur[yi], 1)] = (unsigned short)iR;
    }
    __syncthreads();
    // best right keypoint per left keypoint (:1266-1311)
    const float maxD = prm.mbf / prm.mb, minD = 0.0f;
    const int thOrbDist = (kThHigh + kThLow) / 2;
    for (int iL = t; iL < nL; iL += kStThreads) {
        const plvi_keypoint kp = KL[iL];
        const int row = (int)kp.y;  // vRowIndices[vL] (size_t conversion)
        if (row >= nRows) { atomicOr(err, 1); continue; }
        const int c0 = s_row[row], c1 = s_row[row + 1];
        if (c0 == c1) continue;
        const float minU = kp.x - maxD, maxU = kp.x - minD;
        if (maxU < 0) continue;
        const uint4* ql = reinterpret_cast<const uint4*>(DL + (size_t)iL * 32);
        const uint4 q0 = ql[0], q1 = ql[1];
        unsigned best = ((unsigned)kThHigh << 16) | 0xffffu;
        for (int c = c0; c < c1; ++c) {
            const int iR = s_idx[c];
            const int o = s_roct[iR];
            if (o < kp.octave - 1 || o > kp.octave + 1) continue;
            const float uR = s_rx[iR];
            if (uR >= minU && uR <= maxU) {
                const uint4* qr = reinterpret_cast<const uint4*>(DR + (size_t)iR * 32);
                const uint4 r0 = qr[0], r1 = qr[1];
                const int d = __popc(q0.x ^ r0.x) + __popc(q0.y ^ r0.y) + __popc(q0.z ^ r0.z) + __popc(q0.w ^ r0.w) +
                              __popc(q1.x ^ r1.x) + __popc(q1.y ^ r1.y) + __popc(q1.z ^ r1.z) + __popc(q1.w ^ r1.w);
                const unsigned key = ((unsigned)d << 16) | (unsigned)iR;
                best = key < best ? key : best;
            }
        }
        if ((int)(best >> 16) < thOrbDist) {
            s_res[iL] = (int)(best & 0xffffu);
            s_job[atomicAdd(&s_njob, 1)] = iL;
        }
    }
    __syncthreads();
    // sliding-window SAD + parabola (:1313-1389): one wave per job
    const int njob = s_njob;
    for (int j = wv; j < njob; j += kStThreads / 64) {
        const int iL = s_job[j], iR = s_res[iL];
        const plvi_keypoint kp = KL[iL];
        const int oct = kp.octave;
        const float uR0 = KR[iR].x;
        const float sf = prm.inv[oct];
        const float scaleduL = __builtin_roundf(kp.x * sf);
        const float scaledvL = __builtin_roundf(kp.y * sf);
        const float scaleduR0 = __builtin_roundf(uR0 * sf);
        const int w = 5, L = 5;
        const int lw = lv.w[oct], lh = lv.h[oct];
        const int r0 = (int)(scaledvL - w), c0 = (int)(scaleduL - w);
        const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
        int res = -1;
        if (r0 < 0 || r0 + 2 * w + 1 > lh || c0 < 0 || c0 + 2 * w + 1 > lw) {
            if (lane == 0) atomicOr(err, 2);  // rowRange/colRange assert in the reference
        } else if (!(iniu < 0 || endu >= lw)) {
            const int crLo = (int)(scaleduR0 - L - w);
            if (crLo < 0 || (int)(scaleduR0 + L - w) + 2 * w + 1 > lw) {
                if (lane == 0) atomicOr(err, 2);
            } else {
                const uint8_t* PL = lv.pl[oct] + (size_t)f * lv.planeL[oct];
                const uint8_t* PR = lv.pr[oct] + (size_t)f * lv.planeR[oct];
                const int cL = PL[(size_t)(r0 + w) * lw + c0 + w];
#pragma unroll
                for (int pass = 0; pass < 2; ++pass) {
                    const int p = lane + 64 * pass;
                    if (p < 121) {
                        const int inc = p / 11, ry = p - inc * 11, incR = inc - L;
                        const int cr0 = (int)(scaleduR0 + incR - w);
                        const int cR = PR[(size_t)(r0 + w) * lw + cr0 + w];
                        const uint8_t* rl = PL + (size_t)(r0 + ry) * lw + c0;
                        const uint8_t* rr = PR + (size_t)(r0 + ry) * lw + cr0;
                        int s = 0;
#pragma unroll
                        for (int x = 0; x < 11; ++x) s += abs(((int)rl[x] - cL) - ((int)rr[x] - cR));
                        s_part[wv][p] = s;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane < 11) {
                    int s = 0;
                    for (int ry = 0; ry < 11; ++ry) s += s_part[wv][lane * 11 + ry];
                    s_dist[wv][lane] = s;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) {
                    int bestDist = INT_MAX, bestincR = 0;
                    for (int incR = -L; incR <= L; ++incR) {
                        const float dist = (float)s_dist[wv][incR + L];  // cv::norm(IL, IR, NORM_L1)
                        if (dist < (float)bestDist) {
                            bestDist = (int)dist;
                            bestincR = incR;
                        }
                    }
                    if (bestincR != -L && bestincR != L) {
                        const float dist1 = (float)s_dist[wv][L + bestincR - 1];
                        const float dist2 = (float)s_dist[wv][L + bestincR];
                        const float dist3 = (float)s_dist[wv][L + bestincR + 1];
                        const float deltaR = (dist1 - dist3) / (2.0f * rfmaf(-2.0f, dist2, dist1 + dist3));
                        if (!(deltaR < -1 || deltaR > 1)) {
                            float bestuR = prm.scale[oct] * ((float)scaleduR0 + (float)bestincR + deltaR);
                            float disparity = kp.x - bestuR;
                            if (disparity >= minD && disparity < maxD) {
                                if (disparity <= 0) {
                                    disparity = 0.01f;
                                    bestuR = (float)((double)kp.x - 0.01);
                                }
                                s_dp[iL] = prm.mbf / disparity;
                                s_ur[iL] = bestuR;
                                res = bestDist;
                                atomicAdd(&s_nacc, 1);
                            }
                        }
                    }
                }
            }
        }
        if (lane == 0) s_res[iL] = res;
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // median rejection (:1392-1405): value at sorted position n/2 of the SADs
    const int nacc = s_nacc;
    float thDist = 0.0f;
    if (nacc > 0) {
        const int k = nacc / 2;
        s_hist[t] = 0;
        __syncthreads();
        for (int i = t; i < nL; i += kStThreads)
            if (s_res[i] >= 0) atomicAdd(&s_hist[(s_res[i] >> 8) & 255], 1);  // SAD <= 121*510 < 2^16
        __syncthreads();
        if (t == 0) {
            int c = 0, b = 0;
            while (c + s_hist[b] <= k) c += s_hist[b++];
            s_sel[0] = b;
            s_sel[1] = k - c;
        }
        __syncthreads();
        const int hi = s_sel[0], k2 = s_sel[1];
        s_hist[t] = 0;
        __syncthreads();
        for (int i = t; i < nL; i += kStThreads)
            if (s_res[i] >= 0 && (s_res[i] >> 8) == hi) atomicAdd(&s_hist[s_res[i] & 255], 1);
        __syncthreads();
        if (t == 0) {
            int c = 0, b = 0;
            while (c + s_hist[b] <= k2) c += s_hist[b++];
            s_sel[0] = (hi << 8) | b;
        }
        __syncthreads();
        const float median = (float)s_sel[0];
        const float c15 = 1.5f, c14 = 1.4f;
        thDist = c15 * c14 * median;
    }
    int kept = 0;
    for (int i = t; i < nL; i += kStThreads) {
        float ur = s_ur[i], dp = s_dp[i];
        if (s_res[i] >= 0) {
            if (!((float)s_res[i] < thDist)) ur = dp = -1.0f;
            else kept++;
        }
        uright[(size_t)f * capL + i] = ur;
        depth[(size_t)f * capL + i] = dp;
    }
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
    if (lane == 0) s_tmp[wv] = kept;
    __syncthreads();
    if (t == 0) nstereo[f] = s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3];
}

// ---------------------------------------------------------------------------
// Frame::ComputeStereoMatches_Lines (src/Frame.cc:1408-1492)
// ---------------------------------------------------------------------------
// LineIterator (src/LineIterator.cpp:31-73): calls fn(x, y) for each grid pixel.
template <class Fn>
__device__ __forceinline__ void line_iterate(double x1, double y1, double x2, double y2, Fn fn) {
    const bool steep = fabs(y2 - y1) > fabs(x2 - x1);
    if (steep) { double a = x1; x1 = y1; y1 = a; a = x2; x2 = y2; y2 = a; }
    if (x1 > x2) { double a = x1; x1 = x2; x2 = a; a = y1; y1 = y2; y2 = a; }
    const double dx = x2 - x1, dy = fabs(y2 - y1);
    double error = dx / 2.0;
    const int ystep = (y1 < y2) ? 1 : -1;
    int x = (int)x1, y = (int)y1;
    const int maxX = (int)x2;
    for (; x <= maxX; ++x) {
        if (steep) fn(y, x);
        else fn(x, y);
        error -= dy;
        if (error < 0) { y += ystep; error += dx; }
    }
}

__global__ __launch_bounds__(kStThreads) void stereo_line_grid_kernel(
    const plvi_keyline* __restrict__ klL, const int* __restrict__ nLs, int capL, const plvi_keyline* __restrict__ klR,
    const int* __restrict__ nRs, int capR, double inv_w, double inv_h, int idxCap, int* __restrict__ lines1,
    double* __restrict__ dirs2, int* __restrict__ cell_off, int* __restrict__ cell_idx, int* __restrict__ err) {
    __shared__ int s_cnt[kLGridCells + 1], s_cur[kLGridCells], s_tmp[kStThreads / 64];
    const int f = blockIdx.x, t = threadIdx.x;
    const int nL = nLs[f], nR = nRs[f];
    const plvi_keyline* L = klL + (size_t)f * capL;
    const plvi_keyline* R = klR + (size_t)f * capR;
    int* l1 = lines1 + (size_t)f * capL * 4;
    double* v2 = dirs2 + (size_t)f * capR * 2;
    int* co = cell_off + (size_t)f * (kLGridCells + 1);
    int* ci = cell_idx + (size_t)f * idxCap;
    for (int i = t; i < nL; i += kStThreads) {  // coords (:1422-1426): double products truncated to int
        l1[4 * i] = (int)((double)L[i].startPointX * inv_w);
        l1[4 * i + 1] = (int)((double)L[i].startPointY * inv_h);
        l1[4 * i + 2] = (int)((double)L[i].endPointX * inv_w);
        l1[4 * i + 3] = (int)((double)L[i].endPointY * inv_h);
    }
    for (int i = t; i <= kLGridCells; i += kStThreads) s_cnt[i] = 0;
    for (int i = t; i < kLGridCells; i += kStThreads) s_cur[i] = 0;
    __syncthreads();
    for (int i = t; i < nR; i += kStThreads) {  // directions + grid (:1431-1442)
        const plvi_keyline k = R[i];
        double vx = (double)(k.endPointX - k.startPointX) * inv_w, vy = (double)(k.endPointY - k.startPointY) * inv_h;
        const double m = sqrt(rfma(vx, vx, vy * vy));  // normalize, fused in Frame.cc.o
        vx /= m;
        vy /= m;
        v2[2 * i] = vx;
        v2[2 * i + 1] = vy;
        line_iterate((double)k.startPointX * inv_w, (double)k.startPointY * inv_h, (double)k.endPointX * inv_w,
                     (double)k.endPointY * inv_h, [&](int x, int y) {
                         if (x >= 0 && x < kLGridCols && y >= 0 && y < kLGridRows)
                             atomicAdd(&s_cnt[x * kLGridRows + y], 1);
                     });
    }
    __syncthreads();
    const int total = block_scan_excl(s_cnt, kLGridCells + 1, s_tmp);
    const bool over = total > idxCap;
    for (int i = t; i <= kLGridCells; i += kStThreads) co[i] = over ? 0 : s_cnt[i];
    if (over) {
        if (t == 0) atomicOr(err, 4);
        return;
    }
    for (int i = t; i < nR; i += kStThreads) {
        const plvi_keyline k = R[i];
        line_iterate((double)k.startPointX * inv_w, (double)k.startPointY * inv_h, (double)k.endPointX * inv_w,
                     (double)k.endPointY * inv_h, [&](int x, int y) {
                         if (x >= 0 && x < kLGridCols && y >= 0 && y < kLGridRows) {
                             const int c = x * kLGridRows + y;
                             ci[s_cnt[c] + atomicAdd(&s_cur[c], 1)] = i;
                         }
                     });
    }
    __syncthreads();
    // grid.at(x, y).push_back(idx) in idx order: sort each (short) cell list
    for (int c = t; c < kLGridCells; c += kStThreads) {
        const int a = s_cnt[c], b = s_cnt[c + 1];
        for (int i = a + 1; i < b; ++i) {
            const int v = ci[i];
            int j = i - 1;
            while (j >= a && ci[j] > v) { ci[j + 1] = ci[j]; --j; }
            ci[j + 1] = v;
        }
    }
}

// Frame::lineSegmentOverlapStereo (src/Frame.cc:1494-1529)
__device__ __forceinline__ double dmin(double a, double b) { return b < a ? b : a; }  // std::min
__device__ __forceinline__ double dmax(double a, double b) { return a < b ? b : a; }  // std::max
__device__ double overlap_stereo(double spl_obs, double epl_obs, double spl_proj, double epl_proj) {
    double overlap = 1.f;
    const float lineHorizTh = 0.1f;
    if (fabs(epl_obs - spl_obs) > (double)lineHorizTh) {
        const double sln = dmin(spl_obs, epl_obs), eln = dmax(spl_obs, epl_obs);
        const double spn = dmin(spl_proj, epl_proj), epn = dmax(spl_proj, epl_proj);
        const double length = eln - spn;
        if ((epn < sln) || (spn > eln)) overlap = 0.f;
        else if ((epn > eln) && (spn < sln)) overlap = eln - sln;
        else overlap = dmin(eln, epn) - dmax(sln, spn);
        if (length > (double)0.01f) overlap = overlap / length;
        else overlap = 0.f;
        if (overlap > 1.f) overlap = 1.f;
    }
    return overlap;
}

__global__ __launch_bounds__(kStThreads) void stereo_line_disparity_kernel(
    const plvi_keyline* __restrict__ klL, const int* __restrict__ nLs, int capL, const plvi_keyline* __restrict__ klR,
    const int* __restrict__ nRs, int capR, const plvi_keyline* __restrict__ klUn, float mbf,
    const int* __restrict__ m12, float* __restrict__ disp, float* __restrict__ dep, double* __restrict__ le,
    int* __restrict__ nstereo) {
    const int f = blockIdx.y, i1 = blockIdx.x * kStThreads + threadIdx.x;
    const int nL = nLs[f], nR = nRs[f];
    const size_t o = (size_t)f * capL + i1;
    int ok = 0;
    if (i1 < nL) {
        float ds = -1.0f, de = -1.0f, zs = -1.0f, ze = -1.0f;
        double l0 = 0, l1 = 0, l2 = 0;
        if (nR > 0) {
            const int i2 = m12[o];
            if (i2 >= 0) {
                const plvi_keyline a = klL[o], b = klR[(size_t)f * capR + i2];
                const double spl0 = a.startPointX, spl1 = a.startPointY, epl0 = a.endPointX, epl1 = a.endPointY;
                double spr0 = b.startPointX, spr1 = b.startPointY, epr0 = b.endPointX, epr1 = b.endPointY;
                const double overlap = overlap_stereo(spl1, epl1, spr1, epr1);
                // the left product of each numerator is fused (Frame.cc.o)
                spr0 = rfma(spr0, spl1 - epr1, epr0 * (spr1 - spl1)) / (spr1 - epr1);
                spr1 = spl1;
                epr0 = rfma(spr0, epl1 - epr1, epr0 * (spr1 - epl1)) / (spr1 - epr1);
                epr1 = epl1;
                double disp_s = spl0 - spr0, disp_e = epl0 - epr0;
                const float lsMinDispRatio = 0.7f;
                if (dmin(disp_s, disp_e) / dmax(disp_s, disp_e) < (double)lsMinDispRatio) disp_s = disp_e = -1.0;
                const int minDisp = 1;
                const float lineHorizTh = 0.1f, stereoOverlapTh = 0.75f;
                if (disp_s >= minDisp && disp_e >= minDisp && fabs(spl1 - epl1) > (double)lineHorizTh &&
                    fabs(spr1 - epr1) > (double)lineHorizTh && overlap > (double)stereoOverlapTh) {
                    ds = (float)disp_s;
                    de = (float)disp_e;
                    zs = mbf / (float)disp_s;
                    ze = mbf / (float)disp_e;
                    ok = 1;
                }
            }
            const plvi_keyline u = klUn[o];  // mvle_l (:1486-1491)
            const double a0 = u.startPointX, a1 = u.startPointY, a2 = 1.0, b0 = u.endPointX, b1 = u.endPointY,
                         b2 = 1.0;
            l0 = a1 * b2 - a2 * b1;
            l1 = a2 * b0 - a0 * b2;
            l2 = rfma(a0, b1, -(a1 * b0));  // Eigen cross + norm, fused in Frame.cc.o
            const double s = sqrt(rfma(l0, l0, l1 * l1));
            l0 = l0 / s;
            l1 = l1 / s;
            l2 = l2 / s;
        }
        disp[2 * o] = ds;
        disp[2 * o + 1] = de;
        dep[2 * o] = zs;
        dep[2 * o + 1] = ze;
        le[3 * o] = l0;
        le[3 * o + 1] = l1;
        le[3 * o + 2] = l2;
    }
    ok = __popcll(__ballot(ok));
    if ((threadIdx.x & 63) == 0 && ok) atomicAdd(&nstereo[f], ok);
}

static size_t stereo_orb_lds(int nRows, int capL, int capR, int rowCap) {
    return (size_t)(2 * nRows + 1) * 4 + (size_t)capR * 8 + (size_t)capL * 16 + ((size_t)rowCap * 2 + 15) / 16 * 16;
}

// Launch over raw device tables (shared by the handle and host entry points).
static int launch_stereo_orb(int n, const plvi_keypoint* kL, const uint8_t* dL, const int* nL, int capL,
                             const plvi_keypoint* kR, const uint8_t* dR, const int* nR, int capR,
                             const StereoLv& lv, StereoPrm prm, float* ur, float* dp, int* ns,
                             int* err, hipStream_t st) {
    if (n <= 0) return PLVI_OK;
    if (capL < 1 || capR < 1 || capR > 65535 || prm.nlevels < 1 || prm.nlevels > 16) return PLVI_E_BADARG;
    const float rmax = 2.0f * prm.scale[prm.nlevels - 1];
    prm.rowCap = capR * ((int)std::ceil(2 * rmax) + 3);
    const size_t lds = stereo_orb_lds(lv.h[0], capL, capR, prm.rowCap);
    if (lds > 150 * 1024) return PLVI_E_BADARG;
    hipLaunchKernelGGL(stereo_orb_kernel, dim3(n), dim3(kStThreads), lds, st, kL, dL, nL, capL, kR, dR, nR, capR,
                       lv, prm, ur, dp, ns, err);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_stereo_match_batch(plvi_orb_extractor* left, plvi_orb_extractor* right, int n_frames, float mb,
                                       float mbf, float* d_uright, float* d_depth, int* d_nstereo, int* d_err,
                                       void* stream) {
    if (!left || !right || n_frames < 0 || !(mb > 0)) return PLVI_E_BADARG;
    plvi_keypoint *kL = nullptr, *kR = nullptr;
    uint8_t *dL = nullptr, *dR = nullptr;
    int *nL = nullptr, *nR = nullptr, capL = 0, capR = 0;
    int rc = plvi_orb_outputs(left, &kL, &dL, &nL, nullptr, &capL);
    if (!rc) rc = plvi_orb_outputs(right, &kR, &dR, &nR, nullptr, &capR);
    if (rc) return rc;
    StereoLv lv{};
    StereoPrm prm{};
    prm.mb = mb;
    prm.mbf = mbf;
    float inv[16], sc[16];
    int nlev = 0;
    rc = plvi_orb_pyramid_device(left, -1, nullptr, nullptr, nullptr, nullptr, &nlev);
    if (rc) return rc;
    if (nlev < 1 || nlev > 16) return PLVI_E_BADARG;
    for (int l = 0; l < nlev; ++l) {
        const uint8_t *pl = nullptr, *pr = nullptr;
        size_t fsl = 0, fsr = 0;
        int wl, hl, wr, hr;
        if ((rc = plvi_orb_pyramid_device(left, l, &pl, &fsl, &wl, &hl, nullptr))) return rc;
        if ((rc = plvi_orb_pyramid_device(right, l, &pr, &fsr, &wr, &hr, nullptr))) return rc;
        if (wl != wr || hl != hr) return PLVI_E_BADARG;  // same extractor geometry both sides
        lv.pl[l] = pl;
        lv.pr[l] = pr;
        lv.planeL[l] = (long long)fsl;
        lv.planeR[l] = (long long)fsr;
        lv.w[l] = wl;
        lv.h[l] = hl;
    }
    if ((rc = plvi_orb_scale_tables(left, sc, inv, nullptr, nullptr))) return rc;
    prm.nlevels = nlev;
    for (int l = 0; l < nlev; ++l) { prm.scale[l] = sc[l]; prm.inv[l] = inv[l]; }
    return launch_stereo_orb(n_frames, kL, dL, nL, capL, kR, dR, nR, capR, lv, prm, d_uright, d_depth,
                             d_nstereo, d_err, (hipStream_t)stream);
}

extern "C" int plvi_stereo_match(const plvi_keypoint* kpsL, const uint8_t* descL, int nL, const plvi_keypoint* kpsR,
                                 const uint8_t* descR, int nR, int nlevels, const float* scale, const float* inv_scale,
                                 const uint8_t* pyrL, const uint8_t* pyrR, const long long* lvl_off, const int* lvl_w,
                                 const int* lvl_h, float mb, float mbf, float* uright, float* depth) {
    if (nL < 0 || nR < 0 || nlevels < 1 || nlevels > 16 || !(mb > 0) || !pyrL || !pyrR) return PLVI_E_BADARG;
    if (nL == 0) return 0;
    StereoLv lv{};
    StereoPrm prm{};
    prm.mb = mb;
    prm.mbf = mbf;
    prm.nlevels = nlevels;
    size_t pyrBytes = 0;
    for (int l = 0; l < nlevels; ++l) {
        lv.planeL[l] = lv.planeR[l] = 0;
        lv.w[l] = lvl_w[l];
        lv.h[l] = lvl_h[l];
        prm.scale[l] = scale[l];
        prm.inv[l] = inv_scale[l];
        pyrBytes = std::max(pyrBytes, (size_t)lvl_off[l] + (size_t)lvl_w[l] * lvl_h[l]);
    }
    const int capR = std::max(nR, 1);
    const size_t oKL = 0, oKR = oKL + (size_t)nL * 28, oDL = (oKR + (size_t)capR * 28 + 15) / 16 * 16,
                 oDR = oDL + (size_t)nL * 32, oPL = oDR + (size_t)capR * 32, oPR = oPL + (pyrBytes + 15) / 16 * 16,
                 oO = oPR + (pyrBytes + 15) / 16 * 16, oI = oO + (size_t)nL * 8, total = oI + 16;
    DevBuf d;
    if (d.alloc(total)) return PLVI_E_HIP;
    uint8_t* b = d.as<uint8_t>();
    int* I = reinterpret_cast<int*>(b + oI);  // nL, nR, nstereo, err
    const int counts[4] = {nL, nR, 0, 0};
    PLVI_CHECK(hipMemcpy(b + oKL, kpsL, (size_t)nL * 28, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(b + oDL, descL, (size_t)nL * 32, hipMemcpyHostToDevice));
    if (nR) {
        PLVI_CHECK(hipMemcpy(b + oKR, kpsR, (size_t)nR * 28, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(b + oDR, descR, (size_t)nR * 32, hipMemcpyHostToDevice));
    }
    PLVI_CHECK(hipMemcpy(b + oPL, pyrL, pyrBytes, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(b + oPR, pyrR, pyrBytes, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(I, counts, 16, hipMemcpyHostToDevice));
    for (int l = 0; l < nlevels; ++l) {
        lv.pl[l] = b + oPL + lvl_off[l];
        lv.pr[l] = b + oPR + lvl_off[l];
    }
    float* ur = reinterpret_cast<float*>(b + oO);
    int rc = launch_stereo_orb(1, reinterpret_cast<plvi_keypoint*>(b + oKL), b + oDL, I, nL,
                               reinterpret_cast<plvi_keypoint*>(b + oKR), b + oDR, I + 1, capR, lv,
                               prm, ur, ur + nL, I + 2, I + 3, nullptr);
    if (rc) return rc;
    int out[2];
    PLVI_CHECK(hipMemcpy(uright, ur, (size_t)nL * 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(depth, ur + nL, (size_t)nL * 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(out, I + 2, 8, hipMemcpyDeviceToHost));
    if (out[1]) return PLVI_E_OVERFLOW;
    return out[0];
}

extern "C" size_t plvi_stereo_lines_scratch_bytes(int n_frames, int capL, int capR, int idx_cap) {
    return (size_t)n_frames * ((size_t)capL * 4 * 4 + (size_t)capR * 16 + (size_t)(kLGridCells + 1) * 4 +
                               (size_t)idx_cap * 4 + (size_t)capL * 4 * 4) +
           64;
}

extern "C" int plvi_stereo_lines_batch(int n_frames, const plvi_keyline* d_klL, const uint8_t* d_descL,
                                       const int* d_nL, int capL, const plvi_keyline* d_klR, const uint8_t* d_descR,
                                       const int* d_nR, int capR, const plvi_keyline* d_klUn, int width, int height,
                                       float mbf, int libstdcxx_range_hint, int idx_cap, void* d_scratch,
                                       size_t scratch_bytes, int* d_matches_12, float* d_disparity, float* d_depth,
                                       double* d_le, int* d_nstereo, int* d_err, void* stream) {
    if (n_frames < 0 || capL < 1 || capR < 1 || width <= 0 || height <= 0 || idx_cap < 1) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    if (!d_scratch || scratch_bytes < plvi_stereo_lines_scratch_bytes(n_frames, capL, capR, idx_cap))
        return PLVI_E_BADARG;
    hipStream_t st = (hipStream_t)stream;
    // scratch: [dirs2 f64 | lines1 | cell_off | cell_idx | matchGrid nmatches]
    uint8_t* s = static_cast<uint8_t*>(d_scratch);
    double* dirs = reinterpret_cast<double*>(s);
    int* lines1 = reinterpret_cast<int*>(dirs + (size_t)n_frames * capR * 2);
    int* co = lines1 + (size_t)n_frames * capL * 4;
    int* ci = co + (size_t)n_frames * (kLGridCells + 1);
    int* nm = ci + (size_t)n_frames * idx_cap;
    const double inv_w = kLGridCols / static_cast<double>(width);   // Frame.cc:208-209
    const double inv_h = kLGridRows / static_cast<double>(height);
    hipLaunchKernelGGL(stereo_line_grid_kernel, dim3(n_frames), dim3(kStThreads), 0, st, d_klL, d_nL, capL, d_klR,
                       d_nR, capR, inv_w, inv_h, idx_cap, lines1, dirs, co, ci, d_err);
    PLVI_CHECK(hipGetLastError());
    int rc = plvi_line_match_grid_batch(n_frames, lines1, d_descL, d_nL, capL, kLGridCols, kLGridRows, co, ci, idx_cap,
                                        d_descR, dirs, d_nR, capR, 7, 0, 2, 2, libstdcxx_range_hint, d_matches_12,
                                        nm, d_err, stream);
    if (rc) return rc;
    PLVI_CHECK(hipMemsetAsync(d_nstereo, 0, (size_t)n_frames * 4, st));
    hipLaunchKernelGGL(stereo_line_disparity_kernel, dim3((capL + kStThreads - 1) / kStThreads, n_frames),
                       dim3(kStThreads), 0, st, d_klL, d_nL, capL, d_klR, d_nR, capR, d_klUn ? d_klUn : d_klL, mbf,
                       d_matches_12, d_disparity, d_depth, d_le, d_nstereo);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_stereo_lines(const plvi_keyline* klL, const uint8_t* descL, int nL, const plvi_keyline* klR,
                                 const uint8_t* descR, int nR, const plvi_keyline* klUn, int width, int height,
                                 float mbf, int libstdcxx_range_hint, int* matches_12, float* disparity, float* depth,
                                 double* le) {
    if (nL < 0 || nR < 0 || nL > 2048 || nR > 2048) return PLVI_E_BADARG;
    if (nL == 0) return 0;
    const int capL = nL, capR = std::max(nR, 1), idxCap = 65536;
    const size_t sb = plvi_stereo_lines_scratch_bytes(1, capL, capR, idxCap);
    const size_t oKL = 0, oKR = (size_t)capL * 68, oKU = oKR + (size_t)capR * 68,
                 oDL = (oKU + (size_t)capL * 68 + 15) / 16 * 16, oDR = oDL + (size_t)capL * 32,
                 oLE = (oDR + (size_t)capR * 32 + 15) / 16 * 16, oF = oLE + (size_t)capL * 24,
                 oI = oF + (size_t)capL * 16, oS = (oI + (size_t)capL * 4 + 64 + 15) / 16 * 16, total = oS + sb;
    DevBuf d;
    if (d.alloc(total)) return PLVI_E_HIP;
    uint8_t* b = d.as<uint8_t>();
    int* I = reinterpret_cast<int*>(b + oI);  // m12[capL] | nL nR nstereo err
    int* cnt = I + capL;
    const int counts[4] = {nL, nR, 0, 0};
    PLVI_CHECK(hipMemcpy(b + oKL, klL, (size_t)nL * 68, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(b + oKU, klUn ? klUn : klL, (size_t)nL * 68, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(b + oDL, descL, (size_t)nL * 32, hipMemcpyHostToDevice));
    if (nR) {
        PLVI_CHECK(hipMemcpy(b + oKR, klR, (size_t)nR * 68, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(b + oDR, descR, (size_t)nR * 32, hipMemcpyHostToDevice));
    }
    PLVI_CHECK(hipMemcpy(cnt, counts, 16, hipMemcpyHostToDevice));
    float* F = reinterpret_cast<float*>(b + oF);
    int rc = plvi_stereo_lines_batch(1, reinterpret_cast<plvi_keyline*>(b + oKL), b + oDL, cnt, capL,
                                     reinterpret_cast<plvi_keyline*>(b + oKR), b + oDR, cnt + 1, capR,
                                     reinterpret_cast<plvi_keyline*>(b + oKU), width, height, mbf,
                                     libstdcxx_range_hint, idxCap, b + oS, sb, I, F, F + 2 * capL,
                                     reinterpret_cast<double*>(b + oLE), cnt + 2, cnt + 3, nullptr);
    if (rc) return rc;
    int out[2];
    PLVI_CHECK(hipMemcpy(matches_12, I, (size_t)nL * 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(disparity, F, (size_t)nL * 8, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(depth, F + 2 * capL, (size_t)nL * 8, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(le, b + oLE, (size_t)nL * 24, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(out, cnt + 2, 8, hipMemcpyDeviceToHost));
    if (out[1]) return PLVI_E_OVERFLOW;
    return out[0];
}
