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
#include "plvi_math.h"

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
        // gives NaN, whose |dot| < 0.75 test is false (candidate kept).  Both
        // are fused in the reference build (LineMatcher.cpp.o matchGrid)
        double vx = (double)(epx - spx), vy = (double)(epy - spy);
        const double mag = __builtin_sqrt(rfma(vx, vx, vy * vy));
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
            const double dt = rfma(vx, V2[2 * i2], vy * V2[2 * i2 + 1]);
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
        if (s_overflow && err) atomicOr(err, 1);
    }
}

// ---------------------------------------------------------------------------
// LineMatcher::SearchByProjection(Frame& CurrentFrame, Frame& LastFrame,
// const GridStructure& grid, th, angth) (src/LineMatcher.cpp:274-372), one
// wave per (current, last) frame pair.  The last frame's lines are walked in
// order (a line whose MapLine has Observations() > 0 blocks its best
// current line for every later one, :335-337); per line, lane 0 projects the
// endpoints (Pinhole::project), builds the candidate std::unordered_set<int>
// exactly as libstdc++ holds it (stl_uset.h) and the lanes scan it in
// parallel: the strict-< first argmin in iteration order, then the angle test
// with the float atan2 overload.  The reference's grid y of the second
// endpoint is uv_ep.x * inv_height (:329), kept.
__global__ __launch_bounds__(64) void line_search_proj_kernel(
    plvi_line_proj_params p, const float* __restrict__ cur_angle_all, const uint8_t* __restrict__ cur_desc_all,
    const uint8_t* __restrict__ cur_blocked_all, const int* __restrict__ cur_n, int cur_cap,
    const int* __restrict__ cell_off_all, const int* __restrict__ cell_idx_all, int idx_cap,
    const uint8_t* __restrict__ flags_all, const float* __restrict__ x3dc_all, const int* __restrict__ oct_all,
    const uint8_t* __restrict__ ml_desc_all, const int* __restrict__ last_n, int last_cap, int* __restrict__ match_all,
    int* __restrict__ nmatch, int* __restrict__ err) {
    __shared__ int s_bkt[kGridBktCap], s_nxt[kGridCandCap], s_key[kGridCandCap], s_cand[kGridCandCap];
    __shared__ unsigned char s_blk[kGridRightCap];
    __shared__ int s_ncand, s_overflow, s_go;
    __shared__ float s_uv[4];
    const int pr = blockIdx.x, lane = threadIdx.x;
    const int nc = min(cur_n[pr], cur_cap), nl = min(last_n[pr], last_cap);
    const float* ANG = cur_angle_all + (size_t)pr * cur_cap;
    const uint8_t* CD = cur_desc_all + (size_t)pr * cur_cap * 32;
    const int cols = p.grid_cols, rows = p.grid_rows;
    const int* CO = cell_off_all + (size_t)pr * ((size_t)cols * rows + 1);
    const int* CI = cell_idx_all + (size_t)pr * idx_cap;
    const uint8_t* FL = flags_all + (size_t)pr * last_cap;
    const float* X3 = x3dc_all + (size_t)pr * last_cap * 6;
    const int* OC = oct_all + (size_t)pr * last_cap;
    const uint8_t* MD = ml_desc_all + (size_t)pr * last_cap * 32;
    int* M = match_all + (size_t)pr * cur_cap;
    for (int i = lane; i < nc; i += 64) {
        s_blk[i] = cur_blocked_all ? cur_blocked_all[(size_t)pr * cur_cap + i] : 0;
        M[i] = -1;
    }
    if (lane == 0) s_overflow = 0;
    __syncthreads();
    int matches = 0;
    for (int i = 0; i < nl; ++i) {
        if (!(FL[i] & 1)) continue;
        if (lane == 0) {
            s_go = 0;
            const float* sp = X3 + 6 * i;
            const float* ep = sp + 3;
            const float invzc_sp = (float)(1.0 / (double)sp[2]), invzc_ep = (float)(1.0 / (double)ep[2]);
            const float usx = p.fx * sp[0] / sp[2] + p.cx, usy = p.fy * sp[1] / sp[2] + p.cy;
            const float uex = p.fx * ep[0] / ep[2] + p.cx, uey = p.fy * ep[1] / ep[2] + p.cy;
            bool ok = !(invzc_sp < 0 || invzc_ep < 0);
            ok = ok && !(usx < p.min_x || usx > p.max_x || uex < p.min_x || uex > p.max_x);
            ok = ok && !(usy < p.min_y || usy > p.max_y || uey < p.min_y || uey > p.max_y);
            // a last-frame octave outside [0, nlevels) has no scale: skip the
            // line and flag it (bit 2) instead of reading past scale_l
            const int oct = ok ? OC[i] : 0;
            if (ok && (oct < 0 || oct >= p.nlevels)) {
                ok = false;
                if (err) atomicOr(err, 2);
            }
            if (ok) {
                int window = (int)floorf(p.th);
                if (p.scale_l[oct] > 1) window = (int)floorf(p.th + p.scale_l[oct]);
                const int pts[4] = {(int)((double)usx * p.inv_w), (int)((double)usy * p.inv_h),
                                    (int)((double)uex * p.inv_w), (int)((double)uex * p.inv_h)};  // sic (:329)
                UsetEmu u;
                uset_init(u, s_bkt, kGridBktCap, s_nxt, s_key, kGridCandCap);
                for (int e = 0; e < 2; ++e) {
                    const int x = pts[2 * e], y = pts[2 * e + 1];
                    const int min_x = max(0, x - window), max_x = min(cols, x + window + 1);
                    const int min_y = max(0, y - window), max_y = min(rows, y + window + 1);
                    for (int x_ = min_x; x_ < max_x; ++x_)
                        for (int y_ = min_y; y_ < max_y; ++y_) {
                            const int c = x_ * rows + y_;
                            uset_insert_range(u, CI + CO[c], CO[c + 1] - CO[c], p.range_hint);
                        }
                }
                int k = 0;
                for (int q = u.head; q >= 0 && k < kGridCandCap; q = u.nxt[q]) s_cand[k++] = u.key[q];
                s_ncand = k;
                if (u.overflow) s_overflow = 1;
                s_uv[0] = usx; s_uv[1] = usy; s_uv[2] = uex; s_uv[3] = uey;
                s_go = k > 0;
            }
        }
        __syncthreads();
        if (!s_go) continue;
        const int K = s_ncand;
        const uint4* pa = reinterpret_cast<const uint4*>(MD + (size_t)i * 32);
        const uint4 a0 = pa[0], a1 = pa[1];
        int b = 256, pos = INT_MAX, idx = -1;
        for (int c = lane; c < K; c += 64) {
            const int i2 = s_cand[c];
            if (i2 < 0 || i2 >= nc || s_blk[i2]) continue;
            const uint4* pb = reinterpret_cast<const uint4*>(CD + (size_t)i2 * 32);
            const uint4 c0 = pb[0], c1 = pb[1];
            const int d = __popc(a0.x ^ c0.x) + __popc(a0.y ^ c0.y) + __popc(a0.z ^ c0.z) + __popc(a0.w ^ c0.w) +
                          __popc(a1.x ^ c1.x) + __popc(a1.y ^ c1.y) + __popc(a1.z ^ c1.z) + __popc(a1.w ^ c1.w);
            if (d < b) {  // lane-local candidates come in iteration order
                b = d;
                pos = c;
                idx = i2;
            }
        }
        for (int sh = 32; sh > 0; sh >>= 1) {
            const int ob = __shfl_xor(b, sh), opos = __shfl_xor(pos, sh), oidx = __shfl_xor(idx, sh);
            if (ob < b || (ob == b && opos < pos)) {
                b = ob;
                pos = opos;
                idx = oidx;
            }
        }
        if (b <= 120 && idx >= 0) {  // TH_HIGH
            float theta = ANG[idx] - plvi_atan2f(s_uv[3] - s_uv[1], s_uv[2] - s_uv[0]);
            if (theta < -M_PI) theta = (float)((double)theta + 2 * M_PI);
            else if (theta > M_PI) theta = (float)((double)theta - 2 * M_PI);
            if (fabsf(theta) < p.angth) {
                if (lane == 0) {
                    M[idx] = i;
                    s_blk[idx] = (FL[i] & 2) ? 1 : 0;
                }
                ++matches;
            }
        }
        __syncthreads();
    }
    if (lane == 0) {
        nmatch[pr] = matches;
        if (s_overflow && err) atomicOr(err, 1);
    }
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_line_search_projection_batch(int n_pairs, const plvi_line_proj_params* p,
                                                 const float* d_cur_angle, const uint8_t* d_cur_desc,
                                                 const uint8_t* d_cur_blocked, const int* d_cur_n, int cur_cap,
                                                 const int* d_cell_off, const int* d_cell_idx, int idx_cap,
                                                 const uint8_t* d_last_flags, const float* d_x3dc,
                                                 const int* d_last_octave, const uint8_t* d_ml_desc,
                                                 const int* d_last_n, int last_cap, int* d_match, int* d_nmatches,
                                                 int* d_err, void* stream) {
    if (!p || n_pairs < 0 || cur_cap < 1 || last_cap < 1 || cur_cap > kGridRightCap || p->grid_cols < 1 ||
        p->grid_rows < 1 || p->nlevels < 1 || p->nlevels > 8)
        return PLVI_E_BADARG;
    if (n_pairs == 0) return PLVI_OK;
    hipLaunchKernelGGL(line_search_proj_kernel, dim3(n_pairs), dim3(64), 0, (hipStream_t)stream, *p, d_cur_angle,
                       d_cur_desc, d_cur_blocked, d_cur_n, cur_cap, d_cell_off, d_cell_idx, idx_cap, d_last_flags,
                       d_x3dc, d_last_octave, d_ml_desc, d_last_n, last_cap, d_match, d_nmatches, d_err);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_line_search_projection(const plvi_line_proj_params* p, const float* cur_angle,
                                           const uint8_t* cur_desc, const uint8_t* cur_blocked, int n_cur,
                                           const int* cell_off, const int* cell_idx, const uint8_t* last_flags,
                                           const float* x3dc, const int* last_octave, const uint8_t* ml_desc,
                                           int n_last, int* match) {
    if (!p || n_cur < 0 || n_last < 0 || n_cur > kGridRightCap || (n_cur > 0 && (!cur_angle || !cur_desc || !match)))
        return PLVI_E_BADARG;
    if (n_cur == 0) return 0;
    const int ncell = p->grid_cols * p->grid_rows;
    const int nidx = std::max(cell_off[ncell], 1), lc = std::max(n_last, 1);
    std::vector<size_t> off;
    size_t tot = 0;
    auto put = [&](size_t bytes) {
        off.push_back(tot);
        tot += (bytes + 255) & ~size_t(255);
        return off.size() - 1;
    };
    const size_t oA = put(4 * (size_t)n_cur), oD = put(32 * (size_t)n_cur), oB = put(n_cur), oCO = put(4 * (size_t)(ncell + 1));
    const size_t oCI = put(4 * (size_t)nidx), oF = put(lc), oX = put(24 * (size_t)lc), oO = put(4 * (size_t)lc);
    const size_t oMD = put(32 * (size_t)lc), oM = put(4 * (size_t)n_cur), oN = put(32);
    DevBuf d;
    if (d.alloc(tot)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    auto up = [&](size_t slot, const void* src, size_t bytes) -> int {
        if (src && bytes) PLVI_CHECK(hipMemcpy(B + off[slot], src, bytes, hipMemcpyHostToDevice));
        return PLVI_OK;
    };
    int rc = up(oA, cur_angle, 4 * (size_t)n_cur) | up(oD, cur_desc, 32 * (size_t)n_cur) |
             up(oCO, cell_off, 4 * (size_t)(ncell + 1)) | up(oCI, cell_idx, 4 * (size_t)cell_off[ncell]);
    if (cur_blocked) rc |= up(oB, cur_blocked, n_cur);
    else PLVI_CHECK(hipMemset(B + off[oB], 0, n_cur));
    if (n_last > 0)
        rc |= up(oF, last_flags, n_last) | up(oX, x3dc, 24 * (size_t)n_last) | up(oO, last_octave, 4 * (size_t)n_last) |
              up(oMD, ml_desc, 32 * (size_t)n_last);
    if (rc) return PLVI_E_HIP;
    int counts[4] = {n_cur, n_last, 0, 0};
    PLVI_CHECK(hipMemcpy(B + off[oN], counts, 16, hipMemcpyHostToDevice));
    int* dN = reinterpret_cast<int*>(B + off[oN]);
    rc = plvi_line_search_projection_batch(1, p, reinterpret_cast<const float*>(B + off[oA]), B + off[oD], B + off[oB],
                                           dN, n_cur, reinterpret_cast<const int*>(B + off[oCO]),
                                           reinterpret_cast<const int*>(B + off[oCI]), nidx, B + off[oF],
                                           reinterpret_cast<const float*>(B + off[oX]),
                                           reinterpret_cast<const int*>(B + off[oO]), B + off[oMD], dN + 1, lc,
                                           reinterpret_cast<int*>(B + off[oM]), dN + 2, dN + 3, nullptr);
    if (rc) return rc;
    PLVI_CHECK(hipDeviceSynchronize());
    int res[2] = {0, 0};
    PLVI_CHECK(hipMemcpy(match, B + off[oM], 4 * (size_t)n_cur, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(res, dN + 2, 8, hipMemcpyDeviceToHost));
    if (res[1]) return PLVI_E_CAPACITY;
    return res[0];
}

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
