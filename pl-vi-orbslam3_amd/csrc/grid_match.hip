// grid_match.hip — LineMatcher::matchGrid (src/LineMatcher.cpp:191-272)
// with GridStructure::get (src/gridStructure.cpp:64-75), batched over
// (left, right) frame pairs: stereo line matching (Frame.cc:1408-1451).
//
// The reference walks the left lines in order; `distances[i2]` /
// `matches_21[i2]` carry state from one left line to the next, so lines are
// processed in order by one wave per pair.  Per line, lane 0 rebuilds the
// candidate set exactly as libstdc++'s std::unordered_set<int> would hold it
// (stl_uset.h: same buckets, same rehashes, same node order) and lists it in
// iteration order; the lanes then evaluate the candidates in parallel (the
// cosine test, the Hamming distance, the strictly-better `distances[i2]`
// update — distinct i2 per line, so no races), and a wave reduction picks
// best / second with the first-in-iteration-order tie rule.  The final
// mutual check runs over the left lines in parallel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <vector>

#include "plvi_common.h"
#include "stl_uset.h"

namespace plvi {

constexpr int kGridCandCap = 1024;   // distinct candidates per left line
constexpr int kGridBktCap = 2400;    // >= bucket count reachable with kGridCandCap keys
constexpr int kGridRightCap = 2048;  // lines per side and pair (distances / matches in LDS)

__global__ __launch_bounds__(64) void line_match_grid_kernel(
    const int* __restrict__ lines1, const uint8_t* __restrict__ desc1, const int* __restrict__ n1s, int cap1,
    int cols, int rows, const int* __restrict__ cell_off, const int* __restrict__ cell_idx, int idx_cap,
    const uint8_t* __restrict__ desc2, const double* __restrict__ dirs2, const int* __restrict__ n2s, int cap2,
    int w0, int w1, int h0, int h1, int range_hint, int* __restrict__ m12_out, int* __restrict__ nmatch,
    int* __restrict__ err) {
    __shared__ int s_bkt[kGridBktCap], s_nxt[kGridCandCap], s_key[kGridCandCap], s_cand[kGridCandCap];
    __shared__ int s_dist[kGridRightCap], s_m21[kGridRightCap], s_m12[kGridRightCap];
    __shared__ int s_ncand, s_overflow;
    const int p = blockIdx.x, lane = threadIdx.x;
    const int n1 = n1s[p], n2 = n2s[p];
    const int* L1 = lines1 + (size_t)p * cap1 * 4;
    const uint8_t* D1 = desc1 + (size_t)p * cap1 * 32;
    const int* CO = cell_off + (size_t)p * ((size_t)cols * rows + 1);
    const int* CI = cell_idx + (size_t)p * idx_cap;
    const uint8_t* D2 = desc2 + (size_t)p * cap2 * 32;
    const double* V2 = dirs2 + (size_t)p * cap2 * 2;
    int* M12 = m12_out + (size_t)p * cap1;
    for (int i = lane; i < n2; i += 64) {
        s_dist[i] = INT_MAX;
        s_m21[i] = -1;
    }
    for (int i = lane; i < n1; i += 64) s_m12[i] = -1;
    if (lane == 0) s_overflow = 0;
    __syncthreads();
    int matches = 0;
    for (int i1 = 0; i1 < n1; ++i1) {
        const int spx = L1[4 * i1], spy = L1[4 * i1 + 1], epx = L1[4 * i1 + 2], epy = L1[4 * i1 + 3];
        if (lane == 0) {
            UsetEmu u;
            uset_init(u, s_bkt, kGridBktCap, s_nxt, s_key, kGridCandCap);
            for (int e = 0; e < 2; ++e) {
                const int x = e ? epx : spx, y = e ? epy : spy;
                const int min_x = max(0, x - w0), max_x = min(cols, x + w1 + 1);
                const int min_y = max(0, y - h0), max_y = min(rows, y + h1 + 1);
                for (int x_ = min_x; x_ < max_x; ++x_)
                    for (int y_ = min_y; y_ < max_y; ++y_) {
                        const int c = x_ * rows + y_;
                        uset_insert_range(u, CI + CO[c], CO[c + 1] - CO[c], range_hint);
                    }
            }
            int k = 0;
            for (int q = u.head; q >= 0 && k < kGridCandCap; q = u.nxt[q]) s_cand[k++] = u.key[q];
            s_ncand = k;
            if (u.overflow) s_overflow = 1;
        }
        __syncthreads();
        const int K = s_ncand;
        // std::pair normalize / dot (LineMatcher.h:44-52): a zero-length line
        // gives NaN, whose |dot| < 0.75 test is false (candidate kept)
        double vx = (double)(epx - spx), vy = (double)(epy - spy);
        const double mag = __builtin_sqrt(vx * vx + vy * vy);
        vx /= mag;
        vy /= mag;
        uint4 a0, a1;
        {
            const uint4* pa = reinterpret_cast<const uint4*>(D1 + (size_t)i1 * 32);
            a0 = pa[0];
            a1 = pa[1];
        }
        int b1 = INT_MAX, pos1 = INT_MAX, idx1 = -1, b2 = INT_MAX;
        for (int c = lane; c < K; c += 64) {
            const int i2 = s_cand[c];
            if (i2 < 0 || i2 >= n2) continue;
            const double dt = vx * V2[2 * i2] + vy * V2[2 * i2 + 1];
            if (__builtin_fabs(dt) < 0.75) continue;
            const uint4* pb = reinterpret_cast<const uint4*>(D2 + (size_t)i2 * 32);
            const uint4 c0 = pb[0], c1 = pb[1];
            const int d = __popc(a0.x ^ c0.x) + __popc(a0.y ^ c0.y) + __popc(a0.z ^ c0.z) + __popc(a0.w ^ c0.w) +
                          __popc(a1.x ^ c1.x) + __popc(a1.y ^ c1.y) + __popc(a1.z ^ c1.z) + __popc(a1.w ^ c1.w);
            if (d < s_dist[i2]) {
                s_dist[i2] = d;
                s_m21[i2] = i1;
            } else {
                continue;
            }
            // lane-local candidates come in iteration order
            if (d < b1) {
                b2 = b1;
                b1 = d;
                pos1 = c;
                idx1 = i2;
            } else if (d < b2) {
                b2 = d;
            }
        }
        for (int s = 32; s > 0; s >>= 1) {
            const int ob1 = __shfl_xor(b1, s), opos = __shfl_xor(pos1, s), oidx = __shfl_xor(idx1, s);
            const int ob2 = __shfl_xor(b2, s);
            const int nb2 = min(min(b2, ob2), max(b1, ob1));
            const bool takeO = ob1 < b1 || (ob1 == b1 && opos < pos1);
            if (takeO) {
                b1 = ob1;
                pos1 = opos;
                idx1 = oidx;
            }
            b2 = nb2;
        }
        if ((double)b1 < (double)b2 * 0.9) {
            if (lane == 0) s_m12[i1] = idx1;
            ++matches;
        }
        __syncthreads();
    }
    // mutual check (:258-268)
    int drop = 0;
    for (int i = lane; i < n1; i += 64) {
        int i2 = s_m12[i];
        if (i2 >= 0 && s_m21[i2] != i) {
            i2 = -1;
            ++drop;
        }
        M12[i] = i2;
    }
    for (int s = 32; s > 0; s >>= 1) drop += __shfl_xor(drop, s);
    if (lane == 0) {
        nmatch[p] = matches - drop;
        if (s_overflow) atomicOr(err, 1);
    }
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_line_match_grid_batch(int n_pairs, const int* d_lines1, const uint8_t* d_desc1, const int* d_n1,
                                          int cap1, int grid_cols, int grid_rows, const int* d_cell_off,
                                          const int* d_cell_idx, int idx_cap, const uint8_t* d_desc2,
                                          const double* d_directions2, const int* d_n2, int cap2, int win_w0,
                                          int win_w1, int win_h0, int win_h1, int libstdcxx_range_hint,
                                          int* d_matches_12, int* d_nmatches, int* d_err, void* stream) {
    if (n_pairs < 0 || cap1 < 1 || cap2 < 1 || cap1 > kGridRightCap || cap2 > kGridRightCap || grid_cols < 1 ||
        grid_rows < 1)
        return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    hipLaunchKernelGGL(line_match_grid_kernel, dim3(n_pairs), dim3(64), 0, (hipStream_t)stream, d_lines1, d_desc1,
                       d_n1, cap1, grid_cols, grid_rows, d_cell_off, d_cell_idx, idx_cap, d_desc2, d_directions2, d_n2,
                       cap2, win_w0, win_w1, win_h0, win_h1, libstdcxx_range_hint, d_matches_12, d_nmatches, d_err);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_line_match_grid(const int* lines1, const uint8_t* desc1, int n1, int grid_cols, int grid_rows,
                                    const int* cell_off, const int* cell_idx, const uint8_t* desc2,
                                    const double* directions2, int n2, int win_w0, int win_w1, int win_h0,
                                    int win_h1, int libstdcxx_range_hint, int* matches_12) {
    if (n1 < 0 || n2 < 0 || n1 > kGridRightCap || n2 > kGridRightCap || grid_cols < 1 || grid_rows < 1)
        return PLVI_E_BADARG;
    if (n1 == 0) return 0;
    const int ncell = grid_cols * grid_rows;
    const int nidx = std::max(cell_off[ncell], 1);
    const int cap2 = std::max(n2, 1);
    // [desc1 | desc2 | dirs2 (f64) | ints: lines1, cell_off, cell_idx, n1, n2, out, nm, err]
    const size_t bD1 = (size_t)n1 * 32, bD2 = (size_t)cap2 * 32, bV = (size_t)cap2 * 16;
    const size_t oV = (bD1 + bD2 + 15) / 16 * 16, oI = oV + bV;
    const size_t nInts = (size_t)n1 * 4 + (ncell + 1) + nidx + 2 + n1 + 2;
    DevBuf d;
    if (d.alloc(oI + nInts * 4)) return PLVI_E_HIP;
    uint8_t* base = d.as<uint8_t>();
    int* I = reinterpret_cast<int*>(base + oI);
    int* dL1 = I;
    int* dCO = dL1 + 4 * n1;
    int* dCI = dCO + ncell + 1;
    int* dN = dCI + nidx;
    int* dOut = dN + 2;
    int* dNm = dOut + n1;
    int* dErr = dNm + 1;
    const int counts[2] = {n1, n2};
    PLVI_CHECK(hipMemcpy(base, desc1, bD1, hipMemcpyHostToDevice));
    if (n2) {
        PLVI_CHECK(hipMemcpy(base + bD1, desc2, (size_t)n2 * 32, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(base + oV, directions2, (size_t)n2 * 16, hipMemcpyHostToDevice));
    }
    PLVI_CHECK(hipMemcpy(dL1, lines1, (size_t)n1 * 16, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(dCO, cell_off, (size_t)(ncell + 1) * 4, hipMemcpyHostToDevice));
    if (cell_off[ncell] > 0) PLVI_CHECK(hipMemcpy(dCI, cell_idx, (size_t)cell_off[ncell] * 4, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(dN, counts, 8, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemset(dErr, 0, 4));
    int rc = plvi_line_match_grid_batch(1, dL1, base, dN, n1, grid_cols, grid_rows, dCO, dCI, nidx, base + bD1,
                                        reinterpret_cast<const double*>(base + oV), dN + 1, cap2, win_w0, win_w1,
                                        win_h0, win_h1, libstdcxx_range_hint, dOut, dNm, dErr, nullptr);
    if (rc) return rc;
    int nm = 0, er = 0;
    PLVI_CHECK(hipMemcpy(matches_12, dOut, (size_t)n1 * 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nm, dNm, 4, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&er, dErr, 4, hipMemcpyDeviceToHost));
    if (er) return PLVI_E_CAPACITY;
    return nm;
}
