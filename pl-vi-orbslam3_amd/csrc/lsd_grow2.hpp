// lsd_grow2.hpp — LSD region growing (lsd.cpp:635-686 inside flsd's seed
// loop, :473-504) with TWO tasks per wave.
//
// lsd_grow_kernel keeps one (frame, octave) task per wave and speculates
// over up to 7 queued points (63 lanes), but the BFS frontier of the thin
// LSD regions is ~2 points, so ~2/3 of the lanes idle while the wave pays
// the full per-round instruction cost (the kernel is issue-bound).  Here the
// two 32-lane halves of a wave run two independent tasks (frames 2k and
// 2k+1): up to 3 queued points (27 lanes) per half and round, the same
// speculate / exact-angle-sequence / verify / commit-prefix round as
// lsd_grow_kernel, with every mask, rank and prefix taken per half.  Each
// half owns its LDS window, USED bits and queue.  Control flow stays uniform
// in the round; the seed scan and block setup run under half-uniform
// predicates (a half that has a block ready waits while the other scans).
// The result per task is identical to the sequential algorithm.
#pragma once

namespace plvi {

constexpr int kG2Pts = 3;  // queued points per block and half (27 lanes)

__device__ __forceinline__ unsigned half_bits(unsigned long long m, int hg) {
    return (unsigned)(m >> (32 * hg));
}

// win_load_rows with the 32 lanes of one half
__device__ __forceinline__ void win_load_rows32(const GrowCtx& g, int r0, int r1, int sl) {
    const int n = (r1 - r0) * g.sw;
    const float* src = g.P + (size_t)r0 * g.sw;
    int i = sl;
    for (; i + 7 * 32 < n; i += 8 * 32) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[i + u * 32];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = i + u * 32, row = r0 + j / g.sw, x = j - (j / g.sw) * g.sw;
            g.win[(row & (g.R - 1)) * g.sw + x] = v[u];
        }
    }
    for (; i < n; i += 32) {
        const int row = r0 + i / g.sw, x = i % g.sw;
        g.win[(row & (g.R - 1)) * g.sw + x] = src[i];
    }
    const int nw = (r1 - r0) * g.wpr;
    for (int k = sl; k < nw; k += 32) {
        const int row = r0 + k / g.wpr, w = k % g.wpr;
        g.bits[(row & (g.R - 1)) * g.wpr + w] = gload_l2(g.gbits + (size_t)row * g.wpr + w);
    }
}

__global__ __launch_bounds__(64) void lsd_grow2_kernel(const LineOctDev* __restrict__ octs,
                                                       const float* __restrict__ pix,
                                                       const float4* __restrict__ seedcs,
                                                       unsigned* __restrict__ gbits_all, size_t gbits_frame,
                                                       unsigned* __restrict__ qspill, size_t qspill_frame,
                                                       double prec, LsdRegion* __restrict__ regs,
                                                       unsigned* __restrict__ regpts, size_t regpts_frame,
                                                       int* __restrict__ nlines, int* __restrict__ err, int R, int QL,
                                                       int nf, int smem_task_words) {
    extern __shared__ __align__(16) unsigned lds_u[];
    __builtin_amdgcn_s_setprio(3);
    const int o = blockIdx.x, nOct = gridDim.x;
    const int lane = threadIdx.x, hg = lane >> 5, sl = lane & 31, hb = 32 * hg;
    const int f = blockIdx.y * 2 + hg;
    const bool live = f < nf;
    const LineOctDev& od = octs[o];
    const int sw = od.sw, sh = od.sh;
    const int fs = live ? f : 0;
    const int task = fs * nOct + o;
    GrowCtx g;
    g.sw = sw; g.sh = sh; g.R = R; g.QL = QL;
    g.wpr = (sw + 31) >> 5;
    g.P = pix + od.soff + (size_t)fs * od.splane;
    const float4* SC = seedcs + od.soff + (size_t)fs * od.splane;
    g.gbits = gbits_all + (size_t)task * gbits_frame;
    g.qglob = qspill + (size_t)task * qspill_frame;
    LsdRegion* outR = regs + (size_t)task * kLsdRawCap;
    unsigned* outP = regpts + (size_t)task * regpts_frame;
    g.bits = (lds_u32*)(lds_u + hg * smem_task_words);  // LDS per half: USED ring | queue | angle ring
    g.qlds = g.bits + R * g.wpr;
    g.win = (lds_f32*)(g.qlds + QL);
    g.wb = 0;
    g.ys = 0;
    if (live)
        for (int i = sl; i < sh * g.wpr; i += 32) g.gbits[i] = 0u;
    vm_drain();
    if (live) win_load_rows32(g, 0, min(R, sh), sl);
    vm_drain();
    __syncthreads();
    const int min_reg = od.min_reg_size;
    const int bp = sl / 9, bk = sl % 9;
    const int kdx = bk % 3 - 1, kdy = bk / 3 - 1;
    const unsigned belowh = (1u << sl) - 1u;
    const int halfR = R / 2;
    // per-half task state (uniform within each half)
    int mode = live ? 0 : 2;  // 0 seed scan, 1 region growth, 2 done
    int y = 0, xb = -32;      // current scan chunk
    unsigned m = 0u;          // unvisited seed candidates of the chunk
    float sclx = 0.f, scly = 0.f;
    int nout = 0, npts = 0;
    bool overflow = false;
    int reg_size = 0, i0 = 0, nb = 0, lanes = 0, start = 0;
    bool need_setup = false;
    float sumdx = 0.f, sumdy = 0.f;
    double reg_angle = 0.0;
    // per-lane block state
    int nx = 0, ny = 0;
    float deg = kNotdefF, cc = 0.f, ss = 0.f;
    unsigned dup = 0u;
    bool inblk = false;
    while (true) {
        // ---- seed scan (flsd's raster loop) and block setup, per half, until
        // every live half has a block of queued points to test
        while (true) {
            if (mode == 0) {
                if (m == 0u) {
                    xb += 32;
                    if (xb >= sw - 1) { xb = 0; ++y; }
                    if (y >= sh - 1) {
                        mode = 2;
                    } else {
                        if (xb == 0) {
                            // slide the window by half its height once y is past its middle
                            while (y >= g.wb + halfR && g.wb + R < sh) {
                                const int r0 = g.wb + R, r1 = min(sh, r0 + halfR);
                                win_load_rows32(g, r0, r1, sl);
                                g.wb += r1 - r0;
                                vm_drain();
                            }
                        }
                        g.ys = y;
                        const int x = xb + sl;
                        const bool cand = x < sw - 1 && !used_get(g, x, y) && deg_at(g, x, y) != kNotdefF;
                        m = half_bits(__ballot(cand), hg);
                        sclx = scly = 0.f;
                        if (cand) {
                            const float4 v = SC[(size_t)y * sw + x];
                            sclx = v.x;
                            scly = v.y;
                        }
                    }
                } else {
                    const int b = __ffs(m) - 1;
                    m &= m - 1u;
                    const int sx = xb + b;
                    const float s0 = __shfl(sclx, hb + b), s1 = __shfl(scly, hb + b);
                    if (!used_get(g, sx, y)) {  // not absorbed by an earlier region of this chunk
                        reg_angle = (double)deg_at(g, sx, y) * kD2R;
                        sumdx = s0;
                        sumdy = s1;
                        if (sl == 0) {
                            used_set(g, sx, y);
                            g.qlds[0] = (unsigned)sx | ((unsigned)y << 16);
                        }
                        reg_size = 1;
                        i0 = 0;
                        mode = 1;
                        need_setup = true;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (mode == 1 && need_setup) {
                if (i0 >= reg_size) {
                    // region complete (lsd.cpp:485-486: small regions stay USED);
                    // region2rect runs in lsd_rect_kernel
                    if (reg_size >= min_reg) {
                        if (nout < kLsdRawCap) {
                            for (int j = sl; j < reg_size; j += 32) outP[npts + j] = q_get(g, j);
                            if (sl == 0) outR[nout] = LsdRegion{npts, reg_size, reg_angle};
                            npts += reg_size;
                            ++nout;
                        } else {
                            overflow = true;
                        }
                    }
                    mode = 0;
                    need_setup = false;
                } else {
                    nb = min(kG2Pts, reg_size - i0);
                    lanes = 9 * nb;
                    inblk = sl < lanes;
                    const unsigned pv = inblk ? q_get(g, i0 + bp) : 0u;
                    const int px = (int)(pv & 0xffffu), py = (int)(pv >> 16);
                    nx = px + kdx;
                    ny = py + kdy;
                    const bool valid = inblk && nx >= 0 && nx < sw && ny >= g.ys && ny < sh;
                    deg = valid ? deg_at(g, nx, ny) : kNotdefF;
                    // lanes of earlier block points that test the same pixel
                    const unsigned q0 = __shfl(pv, hb), q1 = __shfl(pv, hb + 9);
                    dup = 0u;
#pragma unroll
                    for (int p2 = 0; p2 < kG2Pts - 1; ++p2) {
                        const unsigned q2 = p2 == 0 ? q0 : q1;
                        const int ddx = nx - (int)(q2 & 0xffffu) + 1, ddy = ny - (int)(q2 >> 16) + 1;
                        if (p2 < bp && inblk && ddx >= 0 && ddx <= 2 && ddy >= 0 && ddy <= 2)
                            dup |= 1u << (9 * p2 + ddy * 3 + ddx);
                    }
                    cc = ss = 0.f;
                    if (deg != kNotdefF) {  // cos/sin(float(angle)) of lsd.cpp:678-679, from lsd_prep_kernel
                        const float4 cs4 = SC[(size_t)ny * sw + nx];
                        cc = cs4.z;
                        ss = cs4.w;
                    }
                    start = 0;
                    need_setup = false;
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (!__ballot(mode == 0 || (mode == 1 && need_setup))) break;
        }
        if (!__ballot(mode == 1)) break;
        // ---- one speculative round for every growing half
        const bool grow = mode == 1;
        const unsigned fromStart = ~0u << start;
        const bool candl = grow && inblk && sl >= start && deg != kNotdefF && !used_get(g, nx, ny);
        const bool al = candl && is_aligned_deg(deg, reg_angle, prec);
        const bool acc = al && (dup & fromStart) == 0u;
        const unsigned A = half_bits(__ballot(acc), hg);
        const int rank = __popc(A & belowh), mcount = __popc(A);
        // compact the accepted lanes' (cos, sin) to lanes hb + rank
        const int dst = acc ? hb + rank : hb + 31;
        const float ccmp = __int_as_float(__builtin_amdgcn_ds_permute(dst << 2, __float_as_int(cc)));
        const float scmp = __int_as_float(__builtin_amdgcn_ds_permute(dst << 2, __float_as_int(ss)));
        // exact angle sequence of the speculated commits: sequential float sums
        // in the reference's order, prefix t kept by lane hb + t
        const int m0 = __builtin_amdgcn_readlane(mcount, 0), m1 = __builtin_amdgcn_readlane(mcount, 32);
        const int mmax = max(m0, m1);
        float sx2 = sumdx, sy2 = sumdy, pfx = 0.f, pfy = 0.f;
        for (int t = 0; t < mmax; ++t) {
            const float ax = readlane_f(ccmp, t), bx = readlane_f(ccmp, 32 + t);
            const float ay = readlane_f(scmp, t), by = readlane_f(scmp, 32 + t);
            if (t < mcount) {
                sx2 += hg ? bx : ax;
                sy2 += hg ? by : ay;
            }
            if (sl == t) { pfx = sx2; pfy = sy2; }
        }
        const double th = (grow && sl < mcount) ? (double)plvi_fast_atan2(pfy, pfx) * kD2R : 0.0;
        // verify every decision against the angle it really sees
        const double thl = shfl_d(th, hb + (rank > 0 ? rank - 1 : 0));
        const double theta_l = rank > 0 ? thl : reg_angle;
        const bool al2 = candl && (dup & A) == 0u && is_aligned_deg(deg, theta_l, prec);
        const unsigned mism = half_bits(__ballot(al2 != acc), hg) & fromStart;
        unsigned C = 0u;
        int nc = 0;
        if (A == 0u) {
            start = lanes;  // no commit: every remaining decision is final
        } else if (mism == 0u) {
            C = A;
            nc = mcount;
            start = lanes;
        } else {
            const int ls = __ffs(mism) - 1;
            C = A & ((1u << ls) - 1u);
            nc = __popc(C);
            start = ls;  // re-decided exactly next round
        }
        const bool mine = grow && ((C >> sl) & 1u);
        if (mine) {
            used_set(g, nx, ny);
            q_put(g, reg_size + __popc(C & belowh), (unsigned)nx | ((unsigned)ny << 16));
        }
        // global USED bits / queue spill must land before they are read back
        if (__ballot((mine && ny >= g.wb + R) || (grow && reg_size + nc > QL))) vm_drain();
        const int srcl = hb + (nc > 0 ? nc - 1 : 0);
        const float nsx = __shfl(pfx, srcl), nsy = __shfl(pfy, srcl);
        const double nth = shfl_d(th, srcl);
        if (grow && nc > 0) {
            reg_size += nc;
            sumdx = nsx;
            sumdy = nsy;
            reg_angle = nth;
        }
        if (grow && start >= lanes) {
            i0 += nb;
            need_setup = true;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (live && sl == 0) {
        nlines[task] = nout;
        if (overflow) atomicOr(err, 4);
    }
}

}  // namespace plvi
