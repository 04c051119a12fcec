// bow.hip — ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
// (src/ORBmatcher.cc:269-471) + ComputeThreeMaxima (:2304-2345), both the
// single-camera branch (F.Nleft == -1) and the two-camera one (:321-420: a
// best / second pair per camera, the right camera's match taken -- without
// its ratio test (`|| true`, :411) -- only when the left best passed TH_LOW,
// the enclosing `if` of the reference), batched over (KF, F) pairs.
//
// The two FeatureVectors (std::map<NodeId, vector<unsigned>>) arrive as CSR
// arrays sorted by node id.  Each F keypoint lives in exactly one node, so
// shared nodes are independent; the only sequential dependency is inside a
// node (a KF keypoint skips F keypoints already matched by an earlier KF
// keypoint of the same node).  Kernel: one workgroup (4 waves) per pair;
// thread 0 walks the two sorted node lists (the reference's lower_bound
// merge); the waves take shared nodes round-robin and walk each node's KF
// keypoints in order, the lanes evaluating the node's F keypoints in
// parallel (best / second with the reference's strict-< first-wins rule as
// a wave reduction).  Matches and the 30-bin rotation histogram live in
// LDS; ComputeThreeMaxima and the 10 % bin filter run at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "plvi_common.h"

namespace plvi {

constexpr int kBowTHLow = 50, kBowHisto = 30;

struct BowBest {
    int b1, p1, b2;  // best distance, its position in the node's F list, second best
};

__device__ __forceinline__ BowBest bow_combine(BowBest x, BowBest y) {
    BowBest r;
    const bool takeY = y.b1 < x.b1 || (y.b1 == x.b1 && y.p1 < x.p1);
    r.b1 = takeY ? y.b1 : x.b1;
    r.p1 = takeY ? y.p1 : x.p1;
    r.b2 = min(min(x.b2, y.b2), max(x.b1, y.b1));
    return r;
}

__global__ __launch_bounds__(256) void search_by_bow_kernel(
    float nnratio, int check_orientation, int kf_cap, int f_cap, int node_cap, const uint8_t* __restrict__ kf_desc,
    const float* __restrict__ kf_angle, const uint8_t* __restrict__ kf_live, const int* __restrict__ kf_node,
    const int* __restrict__ kf_off, const int* __restrict__ kf_nnodes, const int* __restrict__ kf_idx,
    const uint8_t* __restrict__ f_desc, const float* __restrict__ f_angle, const int* __restrict__ f_n,
    const int* __restrict__ f_node, const int* __restrict__ f_off, const int* __restrict__ f_nnodes,
    const int* __restrict__ f_idx, const int* __restrict__ f_nleft, int* __restrict__ match_kf,
    int* __restrict__ nmatches) {
    extern __shared__ __align__(16) int lds[];
    const int p = blockIdx.x;
    int* s_mk = lds;                                      // [f_cap] matched KF index or -1
    int2* s_pairs = reinterpret_cast<int2*>(lds + f_cap);  // [node_cap] shared (KF node, F node)
    __shared__ int s_hist[kBowHisto], s_npairs, s_count, s_keep[3];
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int nF = f_n[p];
    // F.Nleft (-1: one camera, every keypoint is "left")
    const int nLeft = (f_nleft && f_nleft[p] >= 0) ? f_nleft[p] : 0x7fffffff;
    const uint8_t* KD = kf_desc + (size_t)p * kf_cap * 32;
    const float* KA = kf_angle + (size_t)p * kf_cap;
    const uint8_t* KL = kf_live + (size_t)p * kf_cap;
    const int* KN = kf_node + (size_t)p * node_cap;
    const int* KO = kf_off + (size_t)p * (node_cap + 1);
    const int* KI = kf_idx + (size_t)p * kf_cap;
    const uint8_t* FD = f_desc + (size_t)p * f_cap * 32;
    const float* FA = f_angle + (size_t)p * f_cap;
    const int* FN = f_node + (size_t)p * node_cap;
    const int* FO = f_off + (size_t)p * (node_cap + 1);
    const int* FI = f_idx + (size_t)p * f_cap;
    for (int i = tid; i < nF; i += 256) s_mk[i] = -1;
    if (tid < kBowHisto) s_hist[tid] = 0;
    if (tid == 0) {
        // merge walk with the reference's lower_bound jumps (:289-448)
        const int nK = kf_nnodes[p], nFn = f_nnodes[p];
        int a = 0, b = 0, n = 0;
        while (a < nK && b < nFn) {
            const int ka = KN[a], fb = FN[b];
            if (ka == fb) {
                s_pairs[n++] = make_int2(a, b);
                ++a;
                ++b;
            } else if (ka < fb) {
                int lo = a, hi = nK;
                while (lo < hi) { const int mid = (lo + hi) >> 1; if (KN[mid] < fb) lo = mid + 1; else hi = mid; }
                a = lo;
            } else {
                int lo = b, hi = nFn;
                while (lo < hi) { const int mid = (lo + hi) >> 1; if (FN[mid] < ka) lo = mid + 1; else hi = mid; }
                b = lo;
            }
        }
        s_npairs = n;
        s_count = 0;
    }
    __syncthreads();
    const int npairs = s_npairs;
    for (int q = wv; q < npairs; q += 4) {
        const int2 pr = s_pairs[q];
        const int k0 = KO[pr.x], k1 = KO[pr.x + 1];
        const int f0 = FO[pr.y], nfn = FO[pr.y + 1] - f0;
        for (int a = k0; a < k1; ++a) {
            const int realIdxKF = KI[a];
            if (!KL[realIdxKF]) continue;
            const uint4* dk = reinterpret_cast<const uint4*>(KD + (size_t)realIdxKF * 32);
            const uint4 x0 = dk[0], x1 = dk[1];
            BowBest bb{256, 0x7fffffff, 256}, br{256, 0x7fffffff, 256};  // left / right camera
            for (int j = lane; j < nfn; j += 64) {
                const int realIdxF = FI[f0 + j];
                if (s_mk[realIdxF] >= 0) continue;
                const uint4* df = reinterpret_cast<const uint4*>(FD + (size_t)realIdxF * 32);
                const uint4 y0 = df[0], y1 = df[1];
                const int d = __popc(x0.x ^ y0.x) + __popc(x0.y ^ y0.y) + __popc(x0.z ^ y0.z) + __popc(x0.w ^ y0.w) +
                              __popc(x1.x ^ y1.x) + __popc(x1.y ^ y1.y) + __popc(x1.z ^ y1.z) + __popc(x1.w ^ y1.w);
                // lane-local scan in list order with the reference's update rule
                BowBest& t = realIdxF < nLeft ? bb : br;
                if (d < t.b1) {
                    t.b2 = t.b1;
                    t.b1 = d;
                    t.p1 = j;
                } else if (d < t.b2) {
                    t.b2 = d;
                }
            }
            for (int s = 32; s > 0; s >>= 1) {
                BowBest o;
                o.b1 = __shfl_xor(bb.b1, s);
                o.p1 = __shfl_xor(bb.p1, s);
                o.b2 = __shfl_xor(bb.b2, s);
                bb = bow_combine(bb, o);
                if (nLeft != 0x7fffffff) {
                    o.b1 = __shfl_xor(br.b1, s);
                    o.p1 = __shfl_xor(br.p1, s);
                    o.b2 = __shfl_xor(br.b2, s);
                    br = bow_combine(br, o);
                }
            }
            if (bb.b1 <= kBowTHLow && lane == 0) {
                if ((float)bb.b1 < nnratio * (float)bb.b2) s_mk[FI[f0 + bb.p1]] = realIdxKF;
                // the right camera's best, inside the left TH_LOW test, no ratio test (:404-430)
                if (nLeft != 0x7fffffff && br.b1 <= kBowTHLow) s_mk[FI[f0 + br.p1]] = realIdxKF;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    // rotation histogram (:409-419) and ComputeThreeMaxima + filter (:450-468)
    const float factor = 1.0f / kBowHisto;
    if (check_orientation) {
        for (int i = tid; i < nF; i += 256) {
            const int k = s_mk[i];
            if (k < 0) continue;
            float rot = KA[k] - FA[i];
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == kBowHisto) bin = 0;
            atomicAdd(&s_hist[bin], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kBowHisto; i++) {
                const int s = s_hist[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s;
                    ind3 = i;
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
    }
    int cnt = 0;
    for (int i = tid; i < nF; i += 256) {
        int k = s_mk[i];
        if (k >= 0 && check_orientation) {
            float rot = KA[k] - FA[i];
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == kBowHisto) bin = 0;
            if (bin != s_keep[0] && bin != s_keep[1] && bin != s_keep[2]) k = -1;
        }
        match_kf[(size_t)p * f_cap + i] = k;
        cnt += k >= 0;
    }
    atomicAdd(&s_count, cnt);
    __syncthreads();
    if (tid == 0) nmatches[p] = s_count;
}

static size_t bow_smem(int f_cap, int node_cap) { return (size_t)f_cap * 4 + (size_t)node_cap * 8; }

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_search_by_bow_stereo_batch(int n_pairs, float nnratio, int check_orientation, int kf_cap,
                                               int f_cap, int node_cap, const uint8_t* d_kf_desc,
                                               const float* d_kf_angle, const uint8_t* d_kf_live, const int* d_kf_node,
                                               const int* d_kf_off, const int* d_kf_nnodes, const int* d_kf_idx,
                                               const uint8_t* d_f_desc, const float* d_f_angle, const int* d_f_n,
                                               const int* d_f_node, const int* d_f_off, const int* d_f_nnodes,
                                               const int* d_f_idx, const int* d_f_nleft, int* d_match_kf,
                                               int* d_nmatches, void* stream) {
    if (n_pairs < 0 || kf_cap < 1 || f_cap < 1 || node_cap < 1) return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    const size_t smem = bow_smem(f_cap, node_cap);
    if (smem > 64 * 1024) return PLVI_E_CAPACITY;
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)search_by_bow_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  64 * 1024);
    });
    hipLaunchKernelGGL(search_by_bow_kernel, dim3(n_pairs), dim3(256), smem, (hipStream_t)stream, nnratio,
                       check_orientation, kf_cap, f_cap, node_cap, d_kf_desc, d_kf_angle, d_kf_live, d_kf_node,
                       d_kf_off, d_kf_nnodes, d_kf_idx, d_f_desc, d_f_angle, d_f_n, d_f_node, d_f_off, d_f_nnodes,
                       d_f_idx, d_f_nleft, d_match_kf, d_nmatches);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_search_by_bow_batch(int n_pairs, float nnratio, int check_orientation, int kf_cap, int f_cap,
                                        int node_cap, const uint8_t* d_kf_desc, const float* d_kf_angle,
                                        const uint8_t* d_kf_live, const int* d_kf_node, const int* d_kf_off,
                                        const int* d_kf_nnodes, const int* d_kf_idx, const uint8_t* d_f_desc,
                                        const float* d_f_angle, const int* d_f_n, const int* d_f_node,
                                        const int* d_f_off, const int* d_f_nnodes, const int* d_f_idx,
                                        int* d_match_kf, int* d_nmatches, void* stream) {
    return plvi_search_by_bow_stereo_batch(n_pairs, nnratio, check_orientation, kf_cap, f_cap, node_cap, d_kf_desc,
                                           d_kf_angle, d_kf_live, d_kf_node, d_kf_off, d_kf_nnodes, d_kf_idx, d_f_desc,
                                           d_f_angle, d_f_n, d_f_node, d_f_off, d_f_nnodes, d_f_idx, nullptr,
                                           d_match_kf, d_nmatches, stream);
}

// Single pair from host memory, synchronous.  Returns nmatches (>= 0) or an error.
extern "C" int plvi_search_by_bow_stereo(float nnratio, int check_orientation, const uint8_t* kf_desc,
                                         const float* kf_angle, const uint8_t* kf_live, int kf_n, const int* kf_node,
                                         const int* kf_off, int kf_nnodes, const int* kf_idx, const uint8_t* f_desc,
                                         const float* f_angle, int f_n, const int* f_node, const int* f_off,
                                         int f_nnodes, const int* f_idx, int f_nleft, int* match_kf) {
    if (f_nleft < -1 || f_nleft > f_n) return PLVI_E_BADARG;
    if (kf_n < 0 || f_n < 0 || kf_nnodes < 0 || f_nnodes < 0) return PLVI_E_BADARG;
    if (f_n == 0) return 0;
    const int kf_cap = std::max(kf_n, 1), f_cap = f_n, node_cap = std::max(std::max(kf_nnodes, f_nnodes), 1);
    const int nkf_idx = kf_nnodes ? kf_off[kf_nnodes] : 0, nf_idx = f_nnodes ? f_off[f_nnodes] : 0;
    if (nkf_idx > kf_cap || nf_idx > f_cap) return PLVI_E_BADARG;
    // one device block: [kf_desc | f_desc | kf_angle | f_angle | kf_live | ints...]
    std::vector<int> ints;
    auto put = [&](const int* src, int n, int cap) {
        const size_t at = ints.size();
        ints.resize(at + (size_t)cap, 0);
        if (n > 0) std::copy(src, src + n, ints.begin() + at);
        return at;
    };
    const size_t oKN = put(kf_node, kf_nnodes, node_cap), oKO = put(kf_off, kf_nnodes + 1, node_cap + 1);
    const size_t oKC = put(&kf_nnodes, 1, 1), oKI = put(kf_idx, nkf_idx, kf_cap);
    const size_t oFN = put(f_node, f_nnodes, node_cap), oFO = put(f_off, f_nnodes + 1, node_cap + 1);
    const size_t oFC = put(&f_nnodes, 1, 1), oFI = put(f_idx, nf_idx, f_cap), oFn = put(&f_n, 1, 1);
    const size_t oOut = put(nullptr, 0, f_cap), oCnt = put(nullptr, 0, 1), oNl = put(&f_nleft, 1, 1);
    const size_t bytes8 = (size_t)(kf_cap + f_cap) * 32 + (size_t)(kf_cap + f_cap) * 4 + (size_t)kf_cap;
    const size_t intOff = (bytes8 + 15) / 16 * 16;
    DevBuf d;
    if (d.alloc(intOff + ints.size() * 4)) return PLVI_E_HIP;
    uint8_t* base = d.as<uint8_t>();
    uint8_t* dKD = base;
    uint8_t* dFD = dKD + (size_t)kf_cap * 32;
    float* dKA = reinterpret_cast<float*>(dFD + (size_t)f_cap * 32);
    float* dFA = dKA + kf_cap;
    uint8_t* dKL = reinterpret_cast<uint8_t*>(dFA + f_cap);
    int* dI = reinterpret_cast<int*>(base + intOff);
    if (kf_n) {
        PLVI_CHECK(hipMemcpy(dKD, kf_desc, (size_t)kf_n * 32, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(dKA, kf_angle, (size_t)kf_n * 4, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(dKL, kf_live, (size_t)kf_n, hipMemcpyHostToDevice));
    }
    PLVI_CHECK(hipMemcpy(dFD, f_desc, (size_t)f_n * 32, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(dFA, f_angle, (size_t)f_n * 4, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(dI, ints.data(), ints.size() * 4, hipMemcpyHostToDevice));
    int rc = plvi_search_by_bow_stereo_batch(1, nnratio, check_orientation, kf_cap, f_cap, node_cap, dKD, dKA, dKL,
                                             dI + oKN, dI + oKO, dI + oKC, dI + oKI, dFD, dFA, dI + oFn, dI + oFN,
                                             dI + oFO, dI + oFC, dI + oFI, dI + oNl, dI + oOut, dI + oCnt, nullptr);
    if (rc) return rc;
    int cnt = 0;
    PLVI_CHECK(hipMemcpy(match_kf, dI + oOut, (size_t)f_n * 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&cnt, dI + oCnt, 4, hipMemcpyDeviceToHost));
    return cnt;
}

extern "C" int plvi_search_by_bow(float nnratio, int check_orientation, const uint8_t* kf_desc, const float* kf_angle,
                                  const uint8_t* kf_live, int kf_n, const int* kf_node, const int* kf_off,
                                  int kf_nnodes, const int* kf_idx, const uint8_t* f_desc, const float* f_angle,
                                  int f_n, const int* f_node, const int* f_off, int f_nnodes, const int* f_idx,
                                  int* match_kf) {
    return plvi_search_by_bow_stereo(nnratio, check_orientation, kf_desc, kf_angle, kf_live, kf_n, kf_node, kf_off,
                                     kf_nnodes, kf_idx, f_desc, f_angle, f_n, f_node, f_off, f_nnodes, f_idx, -1,
                                     match_kf);
}
