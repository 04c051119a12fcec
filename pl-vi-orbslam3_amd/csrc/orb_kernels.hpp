// orb_kernels.hpp — HIP/CDNA4 kernels of the ORB extractor
// (ORB_SLAM3::ORBextractor, src/ORBextractor.cc).  Compiled with
// -ffp-contract=off: every float op on the bit-exact path is one IEEE op.
//
// Data layout (HBM): for each pyramid level l a region of B frame planes
// (w_l*h_l bytes each) in four parallel buffers: pyr (level image), blur
// (7x7 sigma-2 blur, the rBRIEF input), score (FAST score or 0) and cand
// (NMS survivor response or 0).  SAT = per (frame, level) int32 summed-area
// table of the candidate indicator over the octree region.
#include <hip/hip_runtime.h>

#include "orb_device.h"
#include "plvi_common.h"
#include "plvi_math.h"

namespace plvi {

// ---------------------------------------------------------------------------
// K1: one pyramid level.  Fused: bilinear resize from level l-1 (or copy of
// the input at l=0), 7x7 fixed-point Gaussian blur (reflect-101), FAST-9/16
// score map.  64x16 output tile + 3-px halo staged in LDS.
//   resize  : cv::resize INTER_LINEAR 8U (ORBextractor.cc:1165)
//   blur    : GaussianBlur(7x7, 2) fixed point, taps k0..k3 (ORBextractor.cc:1115; A.4)
//   score   : cornerScore<16> closed form S-1 if S-1 >= tmin else 0 (A.3)
// ---------------------------------------------------------------------------
constexpr int kTW = 64, kTH = 16, kEW = kTW + 6, kEH = kTH + 6;

__device__ __forceinline__ int fast_S(const uint8_t (*e)[kEW + 2], int cx, int cy) {
    // circle offsets (x,y) of cv::FAST makeOffsets(16)
    const int v = e[cy][cx];
    int d[16];
    d[0] = v - e[cy + 3][cx + 0];
    d[1] = v - e[cy + 3][cx + 1];
    d[2] = v - e[cy + 2][cx + 2];
    d[3] = v - e[cy + 1][cx + 3];
    d[4] = v - e[cy + 0][cx + 3];
    d[5] = v - e[cy - 1][cx + 3];
    d[6] = v - e[cy - 2][cx + 2];
    d[7] = v - e[cy - 3][cx + 1];
    d[8] = v - e[cy - 3][cx + 0];
    d[9] = v - e[cy - 3][cx - 1];
    d[10] = v - e[cy - 2][cx - 2];
    d[11] = v - e[cy - 1][cx - 3];
    d[12] = v - e[cy + 0][cx - 3];
    d[13] = v - e[cy + 1][cx - 3];
    d[14] = v - e[cy + 2][cx - 2];
    d[15] = v - e[cy + 3][cx - 1];
    int mn1[16], mx1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mn1[k] = min(d[k], d[(k + 1) & 15]);
        mx1[k] = max(d[k], d[(k + 1) & 15]);
    }
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mn2[k] = min(mn1[k], mn1[(k + 2) & 15]);
        mx2[k] = max(mx1[k], mx1[(k + 2) & 15]);
    }
    int A = -1000, Bm = 1000;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int mn8 = min(mn2[k], mn2[(k + 4) & 15]);
        int mx8 = max(mx2[k], mx2[(k + 4) & 15]);
        A = max(A, min(mn8, d[(k + 8) & 15]));
        Bm = min(Bm, max(mx8, d[(k + 8) & 15]));
    }
    return max(A, -Bm);
}

template <bool RESIZE>
__global__ __launch_bounds__(256) void orb_level_kernel(
    const uint8_t* __restrict__ src, size_t s_frame, size_t s_row, uint8_t* __restrict__ dst,
    uint8_t* __restrict__ blur, uint8_t* __restrict__ score, int w, int h, size_t d_frame,
    const int* __restrict__ xofs, const short* __restrict__ xa, int xmax, const int* __restrict__ yrow,
    const short* __restrict__ yb, int k0, int k1, int k2, int k3, int tmin) {
    __shared__ uint8_t ext[kEH][kEW + 2];
    __shared__ int hs[kEH][kTW];
    const int f = blockIdx.z;
    const int tx0 = blockIdx.x * kTW, ty0 = blockIdx.y * kTH;
    const uint8_t* S = src + (size_t)f * s_frame;
    for (int i = threadIdx.x; i < kEW * kEH; i += 256) {
        const int ex = i % kEW, ey = i / kEW;
        const int gx = reflect101(tx0 + ex - 3, w), gy = reflect101(ty0 + ey - 3, h);
        int v;
        if (RESIZE) {
            const uint8_t* R0 = S + (size_t)yrow[2 * gy] * s_row;
            const uint8_t* R1 = S + (size_t)yrow[2 * gy + 1] * s_row;
            const int b0 = yb[2 * gy], b1 = yb[2 * gy + 1];
            const int sx = xofs[gx];
            int H0, H1;
            if (gx < xmax) {
                const int a0 = xa[2 * gx], a1 = xa[2 * gx + 1];
                H0 = R0[sx] * a0 + R0[sx + 1] * a1;
                H1 = R1[sx] * a0 + R1[sx + 1] * a1;
            } else {
                H0 = R0[sx] * 2048;
                H1 = R1[sx] * 2048;
            }
            v = (((b0 * (H0 >> 4)) >> 16) + ((b1 * (H1 >> 4)) >> 16) + 2) >> 2;
        } else {
            v = S[(size_t)gy * s_row + gx];
        }
        ext[ey][ex] = (uint8_t)v;
    }
    __syncthreads();
    uint8_t* D = dst + (size_t)f * d_frame;
    for (int i = threadIdx.x; i < kEH * kTW; i += 256) {
        const int ey = i / kTW, cx = i % kTW;
        const uint8_t* e = ext[ey];
        hs[ey][cx] = k0 * (e[cx] + e[cx + 6]) + k1 * (e[cx + 1] + e[cx + 5]) + k2 * (e[cx + 2] + e[cx + 4]) +
                     k3 * e[cx + 3];
    }
    __syncthreads();
    uint8_t* Bl = blur + (size_t)f * d_frame;
    uint8_t* Sc = score + (size_t)f * d_frame;
    for (int i = threadIdx.x; i < kTH * kTW; i += 256) {
        const int cy = i / kTW, cx = i % kTW;
        const int x = tx0 + cx, y = ty0 + cy;
        if (x >= w || y >= h) continue;
        D[(size_t)y * w + x] = ext[cy + 3][cx + 3];
        const unsigned s = (unsigned)(k0 * (hs[cy][cx] + hs[cy + 6][cx]) + k1 * (hs[cy + 1][cx] + hs[cy + 5][cx]) +
                                      k2 * (hs[cy + 2][cx] + hs[cy + 4][cx]) + k3 * hs[cy + 3][cx]);
        Bl[(size_t)y * w + x] = (uint8_t)min((s + 32768u) >> 16, 255u);
        int sc = 0;
        if (x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
            const int Sv = fast_S(ext, cx + 3, cy + 3);
            if (Sv - 1 >= tmin && Sv >= 1) sc = Sv - 1;
        }
        Sc[(size_t)y * w + x] = (uint8_t)sc;
    }
}

// ---------------------------------------------------------------------------
// K2: per-cell FAST non-max suppression with the reference's threshold
// fallback (ORBextractor.cc:808-829): survivors at iniThFAST; if none in the
// cell, survivors at minThFAST.  NMS is cell-local: neighbours outside the
// cell's detection window count as 0 (cv::FAST on the cell ROI).
// One wave per (cell, frame).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool nms_keep(const uint8_t* sc, int ww, int wh, int xx, int yy, int t) {
    const int s = sc[yy * kOrbCellMax + xx];
    if (s == 0 || s < t) return false;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            if (!dx && !dy) continue;
            const int nx = xx + dx, ny = yy + dy;
            int nv = 0;
            if (nx >= 0 && nx < ww && ny >= 0 && ny < wh) {
                nv = sc[ny * kOrbCellMax + nx];
                if (nv < t) nv = 0;
            }
            if (!(s > nv)) return false;
        }
    return true;
}

__global__ __launch_bounds__(64) void orb_cell_nms_kernel(const OrbCellDev* __restrict__ cells,
                                                          const OrbLevelDev* __restrict__ lvs,
                                                          const uint8_t* __restrict__ score,
                                                          uint8_t* __restrict__ cand, int t1, int t2) {
    __shared__ uint8_t sc[kOrbCellMax * kOrbCellMax];
    const OrbCellDev c = cells[blockIdx.x];
    const int f = blockIdx.y;
    const OrbLevelDev& L = lvs[c.level];
    const uint8_t* S = score + L.off + (size_t)f * L.plane;
    uint8_t* C = cand + L.off + (size_t)f * L.plane;
    const int ww = c.x1 - c.x0, wh = c.y1 - c.y0;
    const int lane = threadIdx.x;
    for (int i = lane; i < ww * wh; i += 64) {
        const int yy = i / ww, xx = i % ww;
        sc[yy * kOrbCellMax + xx] = S[(size_t)(c.y0 + yy) * L.w + c.x0 + xx];
    }
    __syncthreads();
    int cnt = 0;
    for (int i = lane; i < ww * wh; i += 64) cnt += nms_keep(sc, ww, wh, i % ww, i / ww, t1) ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    const int t = cnt ? t1 : t2;
    for (int i = lane; i < ww * wh; i += 64) {
        const int yy = i / ww, xx = i % ww;
        const bool k = nms_keep(sc, ww, wh, xx, yy, t);
        C[(size_t)(c.y0 + yy) * L.w + c.x0 + xx] = k ? sc[yy * kOrbCellMax + xx] : 0;
    }
}

// ---------------------------------------------------------------------------
// K3: summed-area table of the candidate indicator over each level's octree
// region [minB, minB+rw) x [minB, minB+rh).  SAT[y][x] = #candidates in
// [0,x) x [0,y) (relative coords), (rw+1) x (rh+1).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void orb_sat_rows_kernel(const OrbLevelDev* __restrict__ lvs,
                                                          const uint8_t* __restrict__ cand, int* __restrict__ sat) {
    const int y = blockIdx.x, l = blockIdx.y, f = blockIdx.z;
    const OrbLevelDev& L = lvs[l];
    if (y > L.rh) return;
    int* row = sat + L.satOff + (size_t)f * L.satPlane + (size_t)y * (L.rw + 1);
    const int lane = threadIdx.x;
    if (y == 0) {
        for (int x = lane; x <= L.rw; x += 64) row[x] = 0;
        return;
    }
    const uint8_t* C = cand + L.off + (size_t)f * L.plane + (size_t)(L.minB + y - 1) * L.w + L.minB;
    if (lane == 0) row[0] = 0;
    int carry = 0;
    for (int x0 = 0; x0 < L.rw; x0 += 64) {
        const int x = x0 + lane;
        int v = (x < L.rw && C[x] != 0) ? 1 : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int n = __shfl_up(v, o);
            if (lane >= o) v += n;
        }
        if (x < L.rw) row[x + 1] = carry + v;
        carry += __shfl(v, 63);
    }
}

__global__ __launch_bounds__(256) void orb_sat_cols_kernel(const OrbLevelDev* __restrict__ lvs,
                                                           int* __restrict__ sat) {
    const int l = blockIdx.y, f = blockIdx.z;
    const OrbLevelDev& L = lvs[l];
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x > L.rw) return;
    const int st = L.rw + 1;
    int* col = sat + L.satOff + (size_t)f * L.satPlane + x;
    int acc = 0;
    int y = 1;
    for (; y + 4 <= L.rh + 1; y += 4) {
        const int a = col[(size_t)y * st], b = col[(size_t)(y + 1) * st], c = col[(size_t)(y + 2) * st],
                  d = col[(size_t)(y + 3) * st];
        acc += a; col[(size_t)y * st] = acc;
        acc += b; col[(size_t)(y + 1) * st] = acc;
        acc += c; col[(size_t)(y + 2) * st] = acc;
        acc += d; col[(size_t)(y + 3) * st] = acc;
    }
    for (; y <= L.rh; ++y) {
        acc += col[(size_t)y * st];
        col[(size_t)y * st] = acc;
    }
}

// ---------------------------------------------------------------------------
// K4: ORBextractor::DistributeOctTree (ORBextractor.cc:537-761) as a list
// emulation over node rectangles.  A node's key set is the set of candidates
// inside its membership rectangle, so DivideNode's vKeys copies are replaced
// by O(1) SAT counts; the std::list order (children pushed to the FRONT in
// n1..n4 order, parent erased), the bNoMore flags, both termination tests
// and the phase-2 (size, node*) sort are reproduced exactly, with the
// canonical creation-order tie-break of SURVEY.md B.1.
// One wave per (level, frame); lane 0 runs the list algorithm.
// Output: per node (list order) its membership rectangle.
// ---------------------------------------------------------------------------
struct OctNodes {
    short *gx0, *gy0, *gx1, *gy1;  // geometry UL=(gx0,gy0) BR=(gx1,gy1)
    short *mx0, *my0, *mx1, *my1;  // membership rectangle (half-open)
    int *cnt, *seq;
    short *nxt, *prv, *freel;
    short *vsz, *vprev;
    unsigned char* nomore;
};

__global__ __launch_bounds__(64) void orb_octree_kernel(const OrbLevelDev* __restrict__ lvs,
                                                        const int* __restrict__ sat, short4* __restrict__ out_rect,
                                                        int* __restrict__ out_cnt, int nodeCapMax, int L,
                                                        int* __restrict__ err) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int l = blockIdx.x, f = blockIdx.y;
    const OrbLevelDev& lv = lvs[l];
    const int C = nodeCapMax;
    OctNodes n;
    {
        int* ip = reinterpret_cast<int*>(smem);
        n.cnt = ip; ip += C;
        n.seq = ip; ip += C;
        short* sp = reinterpret_cast<short*>(ip);
        n.gx0 = sp; sp += C; n.gy0 = sp; sp += C; n.gx1 = sp; sp += C; n.gy1 = sp; sp += C;
        n.mx0 = sp; sp += C; n.my0 = sp; sp += C; n.mx1 = sp; sp += C; n.my1 = sp; sp += C;
        n.nxt = sp; sp += C; n.prv = sp; sp += C; n.freel = sp; sp += C;
        n.vsz = sp; sp += C; n.vprev = sp; sp += C;
        n.nomore = reinterpret_cast<unsigned char*>(sp);
    }
    if (threadIdx.x != 0) return;

    const int* S = sat + lv.satOff + (size_t)f * lv.satPlane;
    const int st = lv.rw + 1, RW = lv.rw, RH = lv.rh;
    auto count = [&](int x0, int y0, int x1, int y1) -> int {
        x0 = max(0, min(x0, RW)); x1 = max(0, min(x1, RW));
        y0 = max(0, min(y0, RH)); y1 = max(0, min(y1, RH));
        if (x0 >= x1 || y0 >= y1) return 0;
        return S[y1 * st + x1] - S[y0 * st + x1] - S[y1 * st + x0] + S[y0 * st + x0];
    };
    const int N = lv.quota;
    int nfree = 0;
    for (int i = C - 1; i >= 0; --i) n.freel[nfree++] = (short)i;
    int head = -1, tail = -1, size = 0, seqc = 0;
    bool overflow = false;
    auto alloc = [&]() -> int {
        if (nfree == 0) { overflow = true; return -1; }
        return n.freel[--nfree];
    };
    auto unlink = [&](int i) {
        const int p = n.prv[i], q = n.nxt[i];
        if (p >= 0) n.nxt[p] = (short)q; else head = q;
        if (q >= 0) n.prv[q] = (short)p; else tail = p;
        n.freel[nfree++] = (short)i;
        --size;
    };
    auto push_front = [&](int i) {
        n.prv[i] = -1; n.nxt[i] = (short)head;
        if (head >= 0) n.prv[head] = (short)i; else tail = i;
        head = i;
        ++size;
    };
    // Initial nodes (ORBextractor.cc:541-583): push_back in order; empty erased.
    for (int i = 0; i < lv.nIni; ++i) {
        const int c = count(lv.rootB[i], 0, lv.rootB[i + 1], RH);
        if (c == 0) continue;
        const int k = alloc();
        if (k < 0) break;
        n.gx0[k] = (short)lv.rootGx[i]; n.gy0[k] = 0; n.gx1[k] = (short)lv.rootGx[i + 1]; n.gy1[k] = (short)RH;
        n.mx0[k] = (short)lv.rootB[i]; n.my0[k] = 0; n.mx1[k] = (short)lv.rootB[i + 1]; n.my1[k] = (short)RH;
        n.cnt[k] = c; n.seq[k] = seqc++; n.nomore[k] = (c == 1);
        n.prv[k] = (short)tail; n.nxt[k] = -1;
        if (tail >= 0) n.nxt[tail] = (short)k; else head = k;
        tail = k;
        ++size;
    }
    int nv = 0;  // entries in vsz (vSizeAndPointerToNode)
    // DivideNode + push_front of non-empty children; records >1-children in vsz.
    auto split = [&](int p, int* nToExpand) {
        const int x0 = n.gx0[p], y0 = n.gy0[p], x1 = n.gx1[p], y1 = n.gy1[p];
        const int halfX = (int)ceilf((float)(x1 - x0) / 2), halfY = (int)ceilf((float)(y1 - y0) / 2);
        const int midX = x0 + halfX, midY = y0 + halfY;
        const int mx0 = n.mx0[p], my0 = n.my0[p], mx1 = n.mx1[p], my1 = n.my1[p];
        for (int q = 0; q < 4; ++q) {
            int cx0, cy0, cx1, cy1, bx0, by0, bx1, by1;
            if (q == 0) { cx0 = x0; cy0 = y0; cx1 = midX; cy1 = midY; bx0 = mx0; by0 = my0; bx1 = min(mx1, midX); by1 = min(my1, midY); }
            else if (q == 1) { cx0 = midX; cy0 = y0; cx1 = x1; cy1 = midY; bx0 = max(mx0, midX); by0 = my0; bx1 = mx1; by1 = min(my1, midY); }
            else if (q == 2) { cx0 = x0; cy0 = midY; cx1 = midX; cy1 = y1; bx0 = mx0; by0 = max(my0, midY); bx1 = min(mx1, midX); by1 = my1; }
            else { cx0 = midX; cy0 = midY; cx1 = x1; cy1 = y1; bx0 = max(mx0, midX); by0 = max(my0, midY); bx1 = mx1; by1 = my1; }
            const int c = count(bx0, by0, bx1, by1);
            if (c == 0) continue;
            const int k = alloc();
            if (k < 0) return;
            n.gx0[k] = (short)cx0; n.gy0[k] = (short)cy0; n.gx1[k] = (short)cx1; n.gy1[k] = (short)cy1;
            n.mx0[k] = (short)bx0; n.my0[k] = (short)by0; n.mx1[k] = (short)bx1; n.my1[k] = (short)by1;
            n.cnt[k] = c; n.seq[k] = seqc++; n.nomore[k] = (c == 1);
            push_front(k);
            if (c > 1) {
                if (nToExpand) ++*nToExpand;
                n.vsz[nv++] = (short)k;
            }
        }
    };
    bool finish = false;
    while (!finish && !overflow) {
        int prevSize = size;
        int nToExpand = 0;
        nv = 0;
        for (int it = head; it >= 0;) {
            const int next = n.nxt[it];
            if (!n.nomore[it]) {
                split(it, &nToExpand);
                if (overflow) break;
                unlink(it);
            }
            it = next;
        }
        if (overflow) break;
        if (size >= N || size == prevSize) {
            finish = true;
        } else if (size + nToExpand * 3 > N) {
            while (!finish && !overflow) {
                prevSize = size;
                const int np = nv;
                for (int i = 0; i < np; ++i) n.vprev[i] = n.vsz[i];
                nv = 0;
                // stable insertion sort by (cnt, seq) ascending
                for (int i = 1; i < np; ++i) {
                    const short v = n.vprev[i];
                    const long long kv = ((long long)n.cnt[v] << 32) | (unsigned)n.seq[v];
                    int j = i - 1;
                    while (j >= 0) {
                        const short u = n.vprev[j];
                        const long long ku = ((long long)n.cnt[u] << 32) | (unsigned)n.seq[u];
                        if (ku <= kv) break;
                        n.vprev[j + 1] = u;
                        --j;
                    }
                    n.vprev[j + 1] = v;
                }
                for (int j = np - 1; j >= 0; --j) {
                    const int p = n.vprev[j];
                    split(p, nullptr);
                    if (overflow) break;
                    unlink(p);
                    if (size >= N) break;
                }
                if (size >= N || size == prevSize) finish = true;
            }
        }
    }
    short4* R = out_rect + ((size_t)f * L + l) * nodeCapMax;
    int cntOut = 0;
    if (!overflow) {
        for (int it = head; it >= 0 && cntOut < lv.nodeCap; it = n.nxt[it]) {
            R[cntOut++] = make_short4(n.mx0[it], n.my0[it], n.mx1[it], n.my1[it]);
        }
        if (size > lv.nodeCap) overflow = true;
    }
    out_cnt[(size_t)f * L + l] = overflow ? 0 : cntOut;
    if (overflow) atomicOr(err, 1);
}

// ---------------------------------------------------------------------------
// K5: "Retain the best point in each node" (ORBextractor.cc:739-758): max
// response, ties -> first in the candidate list order (cell-row-major,
// raster within a cell).  One wave per (node, level, frame).  Output level
// keypoint (x, y, response) in level coordinates.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void orb_node_best_kernel(const OrbLevelDev* __restrict__ lvs,
                                                           const uint8_t* __restrict__ cand,
                                                           const short4* __restrict__ rects,
                                                           const int* __restrict__ rect_cnt, int nodeCapMax, int L,
                                                           float4* __restrict__ lvkp, int kpCapFrame) {
    const int node = blockIdx.x, l = blockIdx.y, f = blockIdx.z;
    const int ncnt = rect_cnt[(size_t)f * L + l];
    if (node >= ncnt) return;
    const OrbLevelDev& lv = lvs[l];
    const short4 r = rects[((size_t)f * L + l) * nodeCapMax + node];
    const uint8_t* Cm = cand + lv.off + (size_t)f * lv.plane;
    const int lane = threadIdx.x;
    const int rx0 = r.x, ry0 = r.y, rx1 = r.z, ry1 = r.w;
    const int wdt = rx1 - rx0;
    unsigned long long best = 0;
    const int total = wdt * (ry1 - ry0);
    for (int i = lane; i < total; i += 64) {
        const int yy = ry0 + i / wdt, xx = rx0 + i % wdt;
        const int resp = Cm[(size_t)(lv.minB + yy) * lv.w + lv.minB + xx];
        if (!resp) continue;
        const unsigned ci = (unsigned)(yy - 3) / (unsigned)lv.hCell, cj = (unsigned)(xx - 3) / (unsigned)lv.wCell;
        const unsigned key = ((ci * (unsigned)lv.nCols + cj) * (unsigned)lv.rh + (unsigned)yy) * (unsigned)lv.rw + (unsigned)xx;
        const unsigned long long pk = ((unsigned long long)resp << 32) | (0xFFFFFFFFu - key);
        best = pk > best ? pk : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o);
        best = other > best ? other : best;
    }
    if (lane == 0) {
        const unsigned key = 0xFFFFFFFFu - (unsigned)(best & 0xFFFFFFFFu);
        const unsigned xx = key % (unsigned)lv.rw;
        const unsigned yy = (key / (unsigned)lv.rw) % (unsigned)lv.rh;
        lvkp[(size_t)f * kpCapFrame + lv.kpOff + node] =
            make_float4((float)(xx + lv.minB), (float)(yy + lv.minB), (float)(best >> 32), 0.f);
    }
}

// ---------------------------------------------------------------------------
// K6: IC_Angle on the level image (ORBextractor.cc:75-102) and rBRIEF on the
// blurred level (computeOrbDescriptor :106-145).  One thread per keypoint.
// cosf/sinf are glibc-faithful (plvi_math.h).
// ---------------------------------------------------------------------------
__constant__ signed char c_pattern[1024] = {
#include "orb_pattern.inc"
};
__constant__ int c_umax[16];

// One wave per keypoint (4 waves per workgroup, grid-stride over the slots):
//  * IC_Angle moments: lanes 0..30 / 32..62 take the disc columns u=-15..15
//    of rows v = 0..7 / 8..15, read straight from the level image (each row
//    one coalesced 31-byte segment); integer sums, so any order is exact.
//  * rBRIEF: the 37x37 neighbourhood of the blurred level (rotated pattern
//    offsets are within +-18) is staged in LDS with row-coalesced loads;
//    lane l evaluates tests l, l+64, l+128, l+192 and one ballot per 64
//    tests yields 8 descriptor bytes directly (test j = byte j/8, bit j%8).
constexpr int kDescR = 18, kDescP = 2 * kDescR + 1, kDescPitch = 40;

__global__ __launch_bounds__(256) void orb_describe_kernel(const OrbLevelDev* __restrict__ lvs, int L,
                                                           const uint8_t* __restrict__ pyr,
                                                           const uint8_t* __restrict__ blur,
                                                           const int* __restrict__ rect_cnt,
                                                           float4* __restrict__ lvkp, uint8_t* __restrict__ lvdesc,
                                                           int kpCapFrame) {
    __shared__ uint8_t patch[4][kDescP * kDescPitch];
    const int f = blockIdx.y;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* P = patch[wv];
    const int half = lane >> 5, u = (lane & 31) - 15;
    for (int slot = blockIdx.x * 4 + wv; slot < kpCapFrame; slot += gridDim.x * 4) {
        int l = 0;
        while (l + 1 < L && slot >= lvs[l + 1].kpOff) ++l;
        const OrbLevelDev& lv = lvs[l];
        const int idx = slot - lv.kpOff;
        if (idx >= rect_cnt[(size_t)f * L + l]) continue;  // wave-uniform
        float4 kp = lvkp[(size_t)f * kpCapFrame + slot];
        const int cx = (int)kp.x, cy = (int)kp.y;  // integer-valued level coords
        const int W = lv.w;
        // ---- IC_Angle (ORBextractor.cc:75-102)
        const uint8_t* center = pyr + lv.off + (size_t)f * lv.plane + (size_t)cy * W + cx;
        int m_01 = 0, m_10 = 0;
        if (u <= 15) {
            if (half == 0) m_10 += u * center[u];
            for (int v = half ? 8 : 1; v <= (half ? 15 : 7); ++v) {
                const int d = c_umax[v];
                if (u >= -d && u <= d) {
                    const int vp = center[u + v * W], vm = center[u - v * W];
                    m_01 += v * (vp - vm);
                    m_10 += u * (vp + vm);
                }
            }
        }
        for (int s2 = 32; s2 > 0; s2 >>= 1) {
            m_01 += __shfl_xor(m_01, s2);
            m_10 += __shfl_xor(m_10, s2);
        }
        const float angle = plvi_fast_atan2((float)m_01, (float)m_10);
        if (lane == 0) {
            kp.w = angle;
            lvkp[(size_t)f * kpCapFrame + slot] = kp;
        }
        // ---- rBRIEF (computeOrbDescriptor, ORBextractor.cc:106-145)
        const uint8_t* Bc = blur + lv.off + (size_t)f * lv.plane + (size_t)(cy - kDescR) * W + (cx - kDescR);
        for (int i = lane; i < kDescP * kDescP; i += 64) {
            const int r = i / kDescP, c = i - r * kDescP;
            P[r * kDescPitch + c] = Bc[(size_t)r * W + c];
        }
        const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
        const float ang = angle * factorPI;
        const float a = plvi_cosf(ang), b = plvi_sinf(ang);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        uint64_t* out = reinterpret_cast<uint64_t*>(lvdesc + ((size_t)f * kpCapFrame + slot) * 32);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = lane + 64 * k;
            const float x0 = c_pattern[4 * j], y0 = c_pattern[4 * j + 1];
            const float x1 = c_pattern[4 * j + 2], y1 = c_pattern[4 * j + 3];
            const int t0 = P[(cv_round_f(x0 * b + y0 * a) + kDescR) * kDescPitch + cv_round_f(x0 * a - y0 * b) + kDescR];
            const int t1 = P[(cv_round_f(x1 * b + y1 * a) + kDescR) * kDescPitch + cv_round_f(x1 * a - y1 * b) + kDescR];
            const unsigned long long m = __ballot(t0 < t1);
            if (lane == 0) out[k] = m;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// K7: output assembly of ORBextractor::operator() (ORBextractor.cc:1102-1149):
// level != 0 coordinates scaled by mvScaleFactor; keypoints with
// lap0 <= x <= lap1 go to slots from the back (stereoIndex--), the rest from
// the front (monoIndex++).  One workgroup per frame.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void orb_assemble_kernel(const OrbLevelDev* __restrict__ lvs, int L,
                                                           const int* __restrict__ rect_cnt,
                                                           const float4* __restrict__ lvkp,
                                                           const uint8_t* __restrict__ lvdesc, int kpCapFrame,
                                                           int lap0, int lap1, plvi_keypoint* __restrict__ okp,
                                                           uint8_t* __restrict__ odesc, int* __restrict__ ocount,
                                                           int* __restrict__ omono) {
    const int f = blockIdx.x;
    __shared__ int s_lvOff[kOrbMaxLevels + 1];
    __shared__ int s_scan[256];
    __shared__ int s_monoBase, s_stereoBase;
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int l = 0; l < L; ++l) {
            s_lvOff[l] = acc;
            acc += rect_cnt[(size_t)f * L + l];
        }
        s_lvOff[L] = acc;
        s_monoBase = 0;
        s_stereoBase = 0;
    }
    __syncthreads();
    const int total = s_lvOff[L];
    for (int base = 0; base < total; base += 256) {
        const int g = base + threadIdx.x;
        int l = 0, isMono = 0;
        float4 kp = make_float4(0, 0, 0, 0);
        int slotInLevel = 0;
        if (g < total) {
            while (g >= s_lvOff[l + 1]) ++l;
            slotInLevel = lvs[l].kpOff + (g - s_lvOff[l]);
            kp = lvkp[(size_t)f * kpCapFrame + slotInLevel];
            if (l != 0) {
                kp.x *= lvs[l].scale;
                kp.y *= lvs[l].scale;
            }
            isMono = (kp.x >= (float)lap0 && kp.x <= (float)lap1) ? 0 : 1;
        }
        s_scan[threadIdx.x] = isMono;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const int v = threadIdx.x >= o ? s_scan[threadIdx.x - o] : 0;
            __syncthreads();
            s_scan[threadIdx.x] += v;
            __syncthreads();
        }
        const int monoBefore = s_scan[threadIdx.x] - isMono;  // exclusive
        const int chunkMono = s_scan[255];
        if (g < total) {
            const int stereoBefore = (threadIdx.x - monoBefore);
            const int slot = isMono ? s_monoBase + monoBefore : total - 1 - (s_stereoBase + stereoBefore);
            plvi_keypoint o;
            o.x = kp.x; o.y = kp.y; o.size = lvs[l].size; o.angle = kp.w; o.response = kp.z;
            o.octave = l; o.class_id = -1;
            okp[(size_t)f * kpCapFrame + slot] = o;
            const uint4* sd = reinterpret_cast<const uint4*>(lvdesc + ((size_t)f * kpCapFrame + slotInLevel) * 32);
            uint4* dd = reinterpret_cast<uint4*>(odesc + ((size_t)f * kpCapFrame + slot) * 32);
            dd[0] = sd[0];
            dd[1] = sd[1];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const int nInChunk = min(256, total - base);
            s_monoBase += chunkMono;
            s_stereoBase += nInChunk - chunkMono;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ocount[f] = total;
        omono[f] = s_monoBase;
    }
}

}  // namespace plvi
