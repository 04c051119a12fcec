// match.hip — batched Hamming matchers.
//
//   knn2      : cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) as used by
//               LineMatcher::matchNNR (src/LineMatcher.cpp:41-61): train rows
//               scanned in ascending order, strict-< insertion into a 2-slot
//               list (batchDistance, OpenCV 4.2 core/src/batch_distance.cpp).
//   distance  : ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:2350-2366)
//               = popcount of the 256-bit XOR.
//
// Kernel: one thread per query row, 256 queries per workgroup; train rows
// are staged through LDS in 256-row chunks and read as wave-uniform
// broadcasts.  VALU-bound: 8 x (v_xor + v_bcnt) per descriptor pair.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <vector>

#include "plvi_common.h"

namespace plvi {

constexpr int kKnnQ = 256;      // queries per workgroup
constexpr int kKnnChunk = 256;  // train rows per LDS chunk

__global__ __launch_bounds__(256) void hamming_knn2_kernel(const uint8_t* __restrict__ q, const int* __restrict__ nq,
                                                           int nq_cap, const uint8_t* __restrict__ t,
                                                           const int* __restrict__ nt, int nt_cap,
                                                           int* __restrict__ idx0, int* __restrict__ d0o,
                                                           int* __restrict__ idx1, int* __restrict__ d1o) {
    __shared__ uint4 tr[kKnnChunk * 2];
    const int pair = blockIdx.y;
    const int nQ = nq[pair], nT = nt[pair];
    const int qi = blockIdx.x * kKnnQ + threadIdx.x;
    if (blockIdx.x * kKnnQ >= nQ) return;
    const bool active = qi < nQ;
    uint32_t a[8];
    {
        const uint4* qp = reinterpret_cast<const uint4*>(q + ((size_t)pair * nq_cap + (active ? qi : 0)) * 32);
        const uint4 x = qp[0], y = qp[1];
        a[0] = x.x; a[1] = x.y; a[2] = x.z; a[3] = x.w; a[4] = y.x; a[5] = y.y; a[6] = y.z; a[7] = y.w;
    }
    int b0 = INT_MAX, b1 = INT_MAX, j0 = -1, j1 = -1;
    const uint4* tp = reinterpret_cast<const uint4*>(t + (size_t)pair * nt_cap * 32);
    for (int base = 0; base < nT; base += kKnnChunk) {
        const int n = min(kKnnChunk, nT - base);
        __syncthreads();
        for (int i = threadIdx.x; i < n * 2; i += 256) tr[i] = tp[(size_t)base * 2 + i];
        __syncthreads();
        for (int j = 0; j < n; ++j) {
            const uint4 x = tr[2 * j], y = tr[2 * j + 1];
            int d = __popc(a[0] ^ x.x) + __popc(a[1] ^ x.y) + __popc(a[2] ^ x.z) + __popc(a[3] ^ x.w) +
                    __popc(a[4] ^ y.x) + __popc(a[5] ^ y.y) + __popc(a[6] ^ y.z) + __popc(a[7] ^ y.w);
            if (d < b1) {
                if (d < b0) {
                    b1 = b0; j1 = j0; b0 = d; j0 = base + j;
                } else {
                    b1 = d; j1 = base + j;
                }
            }
        }
    }
    if (active) {
        const size_t o = (size_t)pair * nq_cap + qi;
        idx0[o] = j0; d0o[o] = b0; idx1[o] = j1; d1o[o] = b1;
    }
}

// LineMatcher::match (LineMatcher.cpp:92-111) over a batch of pairs, given
// the kNN-2 tables of both directions: ratio test (float, DMatch::distance)
// then the mutual check.  One workgroup per pair.
__global__ __launch_bounds__(256) void line_match_finish_kernel(const int* __restrict__ n1, const int* __restrict__ n2,
                                                                int cap1, int cap2, const int* __restrict__ i0_12,
                                                                const int* __restrict__ d0_12,
                                                                const int* __restrict__ d1_12,
                                                                const int* __restrict__ i0_21,
                                                                const int* __restrict__ d0_21,
                                                                const int* __restrict__ d1_21, float nnr,
                                                                int* __restrict__ m12, int* __restrict__ nmatch) {
    __shared__ int s_cnt;
    const int p = blockIdx.x;
    const int a = n1[p], b = n2[p];
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    int local = 0;
    for (int i = threadIdx.x; i < a; i += 256) {
        const size_t o = (size_t)p * cap1 + i;
        int m = -1;
        if (b >= 2 && (float)d0_12[o] < (float)d1_12[o] * nnr) m = i0_12[o];
        if (m >= 0) {
            const size_t q = (size_t)p * cap2 + m;
            const int back = (a >= 2 && (float)d0_21[q] < (float)d1_21[q] * nnr) ? i0_21[q] : -1;
            if (back != i) m = -1;
        }
        m12[o] = m;
        local += m >= 0;
    }
    atomicAdd(&s_cnt, local);
    __syncthreads();
    if (threadIdx.x == 0) nmatch[p] = s_cnt;
}

int launch_knn2(const uint8_t* d_q, const int* d_nq, int nq_cap, const uint8_t* d_t, const int* d_nt, int nt_cap,
                int n_pairs, int* i0, int* d0, int* i1, int* d1, hipStream_t st) {
    if (n_pairs <= 0 || nq_cap <= 0) return PLVI_OK;
    dim3 grid((nq_cap + kKnnQ - 1) / kKnnQ, n_pairs);
    hipLaunchKernelGGL(hamming_knn2_kernel, grid, dim3(256), 0, st, d_q, d_nq, nq_cap, d_t, d_nt, nt_cap, i0, d0, i1,
                       d1);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// Scratch context for the synchronous single-pair entry points.
struct MatchCtx {
    std::mutex mu;
    DevBuf q, t, cnt, out;
    size_t qcap = 0, tcap = 0;
    hipStream_t st = nullptr;
    int ensure(size_t nq, size_t nt) {
        if (!st) PLVI_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        if (nq > qcap) {
            q.~DevBuf(); new (&q) DevBuf();
            out.~DevBuf(); new (&out) DevBuf();
            if (q.alloc(nq * 32) || out.alloc(nq * 4 * sizeof(int))) return PLVI_E_HIP;
            qcap = nq;
        }
        if (nt > tcap) {
            t.~DevBuf(); new (&t) DevBuf();
            if (t.alloc(nt * 32)) return PLVI_E_HIP;
            tcap = nt;
        }
        if (!cnt.p && cnt.alloc(2 * sizeof(int))) return PLVI_E_HIP;
        return PLVI_OK;
    }
};
static MatchCtx g_match;

int knn2_host(const uint8_t* q, int nq, const uint8_t* t, int nt, int* i0, int* d0, int* i1, int* d1) {
    if (nq < 0 || nt < 0 || (nq && !q) || (nt && !t)) return PLVI_E_BADARG;
    if (nq == 0) return PLVI_OK;
    std::lock_guard<std::mutex> lk(g_match.mu);
    int rc = g_match.ensure((size_t)nq, (size_t)std::max(nt, 1));
    if (rc) return rc;
    hipStream_t st = g_match.st;
    int counts[2] = {nq, nt};
    PLVI_CHECK(hipMemcpyAsync(g_match.q.p, q, (size_t)nq * 32, hipMemcpyHostToDevice, st));
    if (nt) PLVI_CHECK(hipMemcpyAsync(g_match.t.p, t, (size_t)nt * 32, hipMemcpyHostToDevice, st));
    PLVI_CHECK(hipMemcpyAsync(g_match.cnt.p, counts, sizeof(counts), hipMemcpyHostToDevice, st));
    int* o = g_match.out.as<int>();
    rc = launch_knn2(g_match.q.as<uint8_t>(), g_match.cnt.as<int>(), nq, g_match.t.as<uint8_t>(),
                     g_match.cnt.as<int>() + 1, std::max(nt, 1), 1, o, o + nq, o + 2 * nq, o + 3 * nq, st);
    if (rc) return rc;
    std::vector<int> h((size_t)4 * nq);
    PLVI_CHECK(hipMemcpyAsync(h.data(), o, h.size() * sizeof(int), hipMemcpyDeviceToHost, st));
    PLVI_CHECK(hipStreamSynchronize(st));
    for (int i = 0; i < nq; ++i) {
        if (i0) i0[i] = h[i];
        if (d0) d0[i] = h[nq + i];
        if (i1) i1[i] = h[2 * nq + i];
        if (d1) d1[i] = h[3 * nq + i];
    }
    return PLVI_OK;
}

}  // namespace plvi

extern "C" int plvi_hamming_knn2_batch(const uint8_t* d_q, const int* d_nq, int nq_cap, const uint8_t* d_t,
                                       const int* d_nt, int nt_cap, int n_pairs, int* d_idx0, int* d_d0, int* d_idx1,
                                       int* d_d1, void* stream) {
    if (!d_q || !d_t || !d_nq || !d_nt || nq_cap < 0 || nt_cap < 0 || n_pairs < 0) return PLVI_E_BADARG;
    return plvi::launch_knn2(d_q, d_nq, nq_cap, d_t, d_nt, nt_cap, n_pairs, d_idx0, d_d0, d_idx1, d_d1,
                             (hipStream_t)stream);
}

extern "C" int plvi_line_match_batch(const uint8_t* d_desc1, const int* d_n1, int cap1, const uint8_t* d_desc2,
                                     const int* d_n2, int cap2, int n_pairs, float nnr, int* d_scratch,
                                     int* d_matches_12, int* d_nmatch, void* stream) {
    if (!d_desc1 || !d_desc2 || !d_n1 || !d_n2 || !d_scratch || !d_matches_12 || !d_nmatch || n_pairs < 0)
        return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    hipStream_t st = (hipStream_t)stream;
    int* s = d_scratch;
    int *i0a = s, *d0a = s + (size_t)n_pairs * cap1, *i1a = s + 2 * (size_t)n_pairs * cap1,
        *d1a = s + 3 * (size_t)n_pairs * cap1;
    int* t = s + 4 * (size_t)n_pairs * cap1;
    int *i0b = t, *d0b = t + (size_t)n_pairs * cap2, *i1b = t + 2 * (size_t)n_pairs * cap2,
        *d1b = t + 3 * (size_t)n_pairs * cap2;
    int rc = plvi::launch_knn2(d_desc1, d_n1, cap1, d_desc2, d_n2, cap2, n_pairs, i0a, d0a, i1a, d1a, st);
    if (rc) return rc;
    rc = plvi::launch_knn2(d_desc2, d_n2, cap2, d_desc1, d_n1, cap1, n_pairs, i0b, d0b, i1b, d1b, st);
    if (rc) return rc;
    hipLaunchKernelGGL(plvi::line_match_finish_kernel, dim3(n_pairs), dim3(256), 0, st, d_n1, d_n2, cap1, cap2, i0a,
                       d0a, d1a, i0b, d0b, d1b, nnr, d_matches_12, d_nmatch);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* idx0, int* d0, int* idx1,
                                 int* d1) {
    return plvi::knn2_host(q, nq, t, nt, idx0, d0, idx1, d1);
}

// LineMatcher::matchNNR (LineMatcher.cpp:41-61) with the std::vector
// semantics of matches_12: resize(n1, -1) keeps the first min(n_prev, n1)
// caller entries, accepted matches overwrite theirs.
extern "C" int plvi_line_match_nnr_inout(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr,
                                         int* matches_12, int n_prev) {
    if (n1 < 0 || n2 < 0 || n_prev < 0 || (n1 > 0 && !matches_12)) return PLVI_E_BADARG;
    if (n1 > 0 && n2 < 2) return PLVI_E_BADARG;  // reference reads matches_[idx][1]
    std::vector<int> i0(n1), d0(n1), i1(n1), d1(n1);
    int rc = plvi::knn2_host(desc1, n1, desc2, n2, i0.data(), d0.data(), i1.data(), d1.data());
    if (rc) return rc;
    for (int i = n_prev; i < n1; ++i) matches_12[i] = -1;
    int matches = 0;
    for (int i = 0; i < n1; ++i) {
        // DMatch::distance is float: (float)d0 < (float)d1 * nnr
        if ((float)d0[i] < (float)d1[i] * nnr) {
            matches_12[i] = i0[i];
            ++matches;
        }
    }
    return matches;
}

extern "C" int plvi_line_match_nnr(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr,
                                   int* matches_12) {
    return plvi_line_match_nnr_inout(desc1, n1, desc2, n2, nnr, matches_12, 0);
}

// LineMatcher::match(desc1, desc2, nnr, matches_12) (LineMatcher.cpp:92-111):
// matches_21 is a fresh vector; matches_12 keeps the caller's entries.
extern "C" int plvi_line_match_inout(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr,
                                     int* matches_12, int n_prev) {
    if (n1 < 0 || n2 < 0 || n_prev < 0 || (n1 > 0 && !matches_12)) return PLVI_E_BADARG;
    std::vector<int> m21(n2 > 0 ? n2 : 1);
    std::vector<int> keep(matches_12, matches_12 + std::min(n_prev, n1));
    int matches = plvi_line_match_nnr_inout(desc1, n1, desc2, n2, nnr, matches_12, n_prev);
    if (matches < 0) return matches;
    int rc = plvi_line_match_nnr(desc2, n2, desc1, n1, nnr, m21.data());
    if (rc < 0) return rc;
    for (int i1 = 0; i1 < n1; ++i1)
        if (matches_12[i1] >= n2) {  // stale entry beyond desc2: undefined in the reference
            std::copy(keep.begin(), keep.end(), matches_12);
            return PLVI_E_BADARG;
        }
    for (int i1 = 0; i1 < n1; ++i1) {
        int& i2 = matches_12[i1];
        if (i2 >= 0 && m21[i2] != i1) {
            i2 = -1;
            --matches;
        }
    }
    return matches;
}

extern "C" int plvi_line_match(const uint8_t* desc1, int n1, const uint8_t* desc2, int n2, float nnr,
                               int* matches_12) {
    return plvi_line_match_inout(desc1, n1, desc2, n2, nnr, matches_12, 0);
}

// ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:2350-2366, per-word
// count >> 24 = popcount) and LineMatcher::DescriptorDistance
// (src/LineMatcher.cpp:487-499, the >> 25 quirk: each word's count halved
// and floored), over n row pairs (a[i], b[i]).
namespace plvi {
__global__ __launch_bounds__(256) void descriptor_distance_kernel(const uint8_t* __restrict__ a,
                                                                  const uint8_t* __restrict__ b, int n, int shift,
                                                                  int* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4* pa = reinterpret_cast<const uint4*>(a + (size_t)i * 32);
    const uint4* pb = reinterpret_cast<const uint4*>(b + (size_t)i * 32);
    const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    const unsigned w[8] = {a0.x ^ b0.x, a0.y ^ b0.y, a0.z ^ b0.z, a0.w ^ b0.w,
                           a1.x ^ b1.x, a1.y ^ b1.y, a1.z ^ b1.z, a1.w ^ b1.w};
    int d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d += (int)((unsigned)__popc(w[k]) >> (shift - 24));
    out[i] = d;
}
}  // namespace plvi

extern "C" int plvi_descriptor_distance_batch(const uint8_t* d_a, const uint8_t* d_b, int n, int line_matcher_quirk,
                                              int* d_out, void* stream) {
    if (n < 0 || (n && (!d_a || !d_b || !d_out))) return PLVI_E_BADARG;
    if (n == 0) return PLVI_OK;
    hipLaunchKernelGGL(plvi::descriptor_distance_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       d_a, d_b, n, line_matcher_quirk ? 25 : 24, d_out);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}
