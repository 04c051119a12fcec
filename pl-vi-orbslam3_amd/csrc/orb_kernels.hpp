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

// reflect-101 for an overshoot of at most len-1 (tile halos are 3 px)
__device__ __forceinline__ int reflect1(int p, int len) {
    p = p < 0 ? -p : p;
    p = p >= len ? 2 * len - 2 - p : p;
    return max(p, 0);
}


// ---------------------------------------------------------------------------
// K1a: ComputePyramid (ORBextractor.cc:1152-1177): levels 1..L-1, chained
// cv::resize INTER_LINEAR 8U (level l from l-1), streamed top to
// bottom in a single launch.  A workgroup holds kPyrFrames frames:
//   wave 0 (loader): streams the level-0 rows of its frames from HBM (dword
//     loads, kPyrAhead rows per frame in flight) into per-frame LDS rings of
//     kPyrRing rows;
//   waves 1..kPyrFrames (resizers, one per frame): every new source row
//     yields the (at most one: scale > 1) next row of the level above it,
//     cascading through the levels; each level keeps its last two rows in
//     LDS, and every level row is written to HBM once -- no intermediate
//     HBM round trip.
// Waves hand rows over through per-frame LDS counters (rows loaded / rows
// consumed) and s_sleep polling, never a workgroup barrier: a resizer issues
// only stores and LDS traffic, so nothing in its loop waits for memory.
// The per-column coefficients (sx, a0, a1 of cv::resize, computed on the
// host exactly as OpenCV does: append_xtab) are one packed table in LDS
// shared by the workgroup's frames; the row coefficients are computed per
// output row.  The fixed-point products use 24-bit multiplies (operands
// < 2^24: pixel x 2048 and (H >> 4) x 2048).
// Limits: level-0 width <= 4 * 64 * kPyrDw, source widths <= 1024.
// ---------------------------------------------------------------------------
#ifndef PLVI_PYR_FRAMES
#define PLVI_PYR_FRAMES 4
#endif
constexpr int kPyrAhead = 2, kPyrDw = 4, kPyrRing = 4, kPyrUnroll = 4, kPyrFrames = PLVI_PYR_FRAMES;

// packed column entry: sx (10 bits) | a0 (12 bits) << 10 | (a0 + a1 - 2047) (2 bits) << 22 | clampR << 24
__host__ __device__ inline uint32_t pyr_xtab_pack(int sx, int a0, int a1, bool clampR) {
    return (uint32_t)sx | ((uint32_t)a0 << 10) | ((uint32_t)(a0 + a1 - 2047) << 22) | ((uint32_t)clampR << 24);
}

// Loader -> resizer hand-off of the pyramid kernel's LDS row ring, inside the
// HIP memory model: the producing wave makes all its lanes' row writes
// visible to its lane 0 (wavefront-scope release / acquire around a wave
// barrier), lane 0 publishes the row counter with a workgroup-scope RELEASE
// store, and the consuming wave polls it with workgroup-scope ACQUIRE loads
// (on gfx950 both compile to an s_waitcnt lgkmcnt(0) for LDS).
__device__ __forceinline__ int lds_load_acquire(lds_i32* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(lds_i32* p, int v, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

#ifndef PLVI_ORB_SETPRIO
#define PLVI_ORB_SETPRIO 0  // s_setprio of the ORB chain's waves (0: hardware default, no instruction)
#endif
#define PLVI_ORB_PRIO_SET()                                                      \
    do {                                                                         \
        if (PLVI_ORB_SETPRIO) __builtin_amdgcn_s_setprio(PLVI_ORB_SETPRIO);      \
    } while (0)
#ifndef PLVI_BF_SETPRIO
#define PLVI_BF_SETPRIO 0  // s_setprio of the blur + FAST waves alone (0: as the ORB chain)
#endif

#ifndef PLVI_PYR_WPE
#define PLVI_PYR_WPE 1  // waves per EU the pyramid kernel is compiled for (1: no cap)
#endif
__global__ __launch_bounds__(64 * (kPyrFrames + 1)) __attribute__((amdgpu_waves_per_eu(PLVI_PYR_WPE))) void orb_pyramid_kernel(
    const OrbLevelDev* __restrict__ lvs, int L, const uint8_t* __restrict__ frames, size_t f_frame, size_t f_row,
    int nf, uint8_t* __restrict__ pyr, const uint32_t* __restrict__ xtab, int xtab_n, int frame_lds, int generic) {
    PLVI_ORB_PRIO_SET();
    extern __shared__ __align__(16) uint8_t lds_pyr_g[];
    __shared__ int s_w[kOrbMaxLevels], s_h[kOrbMaxLevels], s_roff[kOrbMaxLevels], s_xoff[kOrbMaxLevels];
    __shared__ double s_sy[kOrbMaxLevels];
    __shared__ int s_cnt[2 * kPyrFrames];  // per frame: rows loaded, rows consumed
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // uniform: scalar role / frame
    const int f0 = blockIdx.x * kPyrFrames;
    const int nfw = min(kPyrFrames, nf - f0);  // frames of this workgroup
    lds_u32* ltab = (lds_u32*)lds_pyr_g;     // column table first (xtab_n words)
    if (threadIdx.x < L) {
        s_w[threadIdx.x] = lvs[threadIdx.x].w;
        s_h[threadIdx.x] = lvs[threadIdx.x].h;
        s_sy[threadIdx.x] = lvs[threadIdx.x].rsy;
        s_xoff[threadIdx.x] = lvs[threadIdx.x].xtab;
    }
    if (threadIdx.x == 0) {
        int o = kPyrRing * ((lvs[0].w + 3) & ~3);  // level-0 ring first
        s_roff[0] = 0;
        for (int l = 1; l < L - 1; ++l) {
            s_roff[l] = o;
            o += 2 * ((lvs[l].w + 3) & ~3);
        }
    }
    if (threadIdx.x < 2 * kPyrFrames) s_cnt[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < xtab_n; i += 64 * (kPyrFrames + 1)) ltab[i] = xtab[i];
    __syncthreads();  // the only workgroup barrier
    const int W0 = s_w[0], H0 = s_h[0];
    const int pitch0 = (W0 + 3) & ~3;
    lds_u8* fbase = (lds_u8*)(lds_pyr_g + 4 * xtab_n);  // per-frame regions of frame_lds bytes
    if (wave == 0) {
        // ------------------------------------------------ loader
        const int nd = (W0 + 3) >> 2;
        bool al4 = (W0 & 3) == 0 && (f_row & 3) == 0 && (f_frame & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(frames) & 3) == 0;
        auto load_row = [&](int k, int r, uint32_t* v) {
            const uint8_t* row = frames + (size_t)(f0 + k) * f_frame + (size_t)r * f_row;
            if (al4) {
                const uint32_t* rw = reinterpret_cast<const uint32_t*>(row);
#pragma unroll
                for (int q = 0; q < kPyrDw; ++q)
                    v[q] = lane + 64 * q < nd ? __builtin_nontemporal_load(rw + lane + 64 * q) : 0u;
            } else {
#pragma unroll
                for (int q = 0; q < kPyrDw; ++q) {
                    const int d = lane + 64 * q;
                    uint32_t x = 0;
                    for (int b = 0; b < 4; ++b)
                        if (4 * d + b < W0) x |= (uint32_t)row[4 * d + b] << (8 * b);
                    v[q] = x;
                }
            }
        };
        uint32_t pf[kPyrAhead][kPyrFrames][kPyrDw];
#pragma unroll
        for (int j = 0; j < kPyrAhead; ++j)
#pragma unroll
            for (int k = 0; k < kPyrFrames; ++k)
                if (j < H0 && k < nfw) load_row(k, j, pf[j][k]);
        for (int rb = 0; rb < H0; rb += kPyrAhead) {
#pragma unroll
            for (int j = 0; j < kPyrAhead; ++j) {
                const int r = rb + j;
                if (r >= H0) break;
#pragma unroll
                for (int k = 0; k < kPyrFrames; ++k) {
                    if (k >= nfw) break;
                    lds_i32* loaded = (lds_i32*)&s_cnt[2 * k];
                    lds_i32* consumed = (lds_i32*)&s_cnt[2 * k + 1];
                    // the resizer needs rows consumed-1 and consumed: slot r % ring is free once r - ring <= consumed - 2
                    while (r - kPyrRing > lds_load_acquire(consumed) - 2) __builtin_amdgcn_s_sleep(1);
                    lds_u32* slot = (lds_u32*)(fbase + (size_t)k * frame_lds + (r % kPyrRing) * pitch0);
#pragma unroll
                    for (int q = 0; q < kPyrDw; ++q)
                        if (lane + 64 * q < nd) slot[lane + 64 * q] = pf[j][k][q];
                    lds_publish(loaded, r + 1, lane);
                    if (r + kPyrAhead < H0) load_row(k, r + kPyrAhead, pf[j][k]);
                }
            }
        }
        return;
    }
    // ---------------------------------------------------- resizer of frame f
    const int k = wave - 1;
    if (k >= nfw) return;
    const int f = f0 + k;
    lds_u8* lds_pyr = fbase + (size_t)k * frame_lds;
    lds_i32* s_loaded = (lds_i32*)&s_cnt[2 * k];
    lds_i32* s_consumed = (lds_i32*)&s_cnt[2 * k + 1];
    // this frame's level planes (no global parameter loads inside the row loop)
    uint8_t* dbase[kOrbMaxLevels];
#pragma unroll
    for (int l = 0; l < kOrbMaxLevels; ++l)
        dbase[l] = l < L ? pyr + lvs[l].off + (size_t)f * lvs[l].plane : nullptr;
    int prod[kOrbMaxLevels];
#pragma unroll
    for (int l = 0; l < kOrbMaxLevels; ++l) prod[l] = 0;
    for (int r = 0; r < H0; ++r) {
        while (lds_load_acquire(s_loaded) <= r) __builtin_amdgcn_s_sleep(1);
        int avail = r + 1;  // rows of the source level available
        for (int l = 1; l < L; ++l) {
            const int sh = s_h[l - 1], w = s_w[l], h = s_h[l];
            const int spitch = (s_w[l - 1] + 3) & ~3, pitch = (w + 3) & ~3;
            const int sring = l == 1 ? kPyrRing : 2;
            const double scy = s_sy[l];
            const lds_u32* T = ltab + s_xoff[l];
            int y = prod[l];
            const int y_start = y;
            while (y < h) {
                float fy = (float)((y + 0.5) * scy - 0.5);
                int sy = (int)fy;
                sy -= (sy > fy);
                fy -= (float)sy;
                const int r1 = min(max(sy + 1, 0), sh - 1);
                if (r1 >= avail) break;
                const int r0 = min(max(sy, 0), sh - 1);
                const unsigned b0 = (unsigned)__builtin_rintf((1.f - fy) * 2048),
                               b1 = (unsigned)__builtin_rintf(fy * 2048);
                const lds_u8* S0 = lds_pyr + s_roff[l - 1] + (r0 % sring) * spitch;
                const lds_u8* S1 = lds_pyr + s_roff[l - 1] + (r1 % sring) * spitch;
                uint8_t* D = dbase[l] + (size_t)y * w;
                lds_u8* R = l < L - 1 ? lds_pyr + s_roff[l] + (y & 1) * pitch : nullptr;
                for (int x0 = 0; x0 < w; x0 += 64 * kPyrUnroll) {
                    // kPyrUnroll columns per lane: all LDS reads issued before the first use
                    uint32_t e[kPyrUnroll];
                    unsigned p00[kPyrUnroll], p01[kPyrUnroll], p10[kPyrUnroll], p11[kPyrUnroll];
#pragma unroll
                    for (int u = 0; u < kPyrUnroll; ++u) {
                        const int x = x0 + 64 * u + lane;
                        e[u] = x < w ? T[x] : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < kPyrUnroll; ++u) {
                        const int sx = e[u] & 1023;
                        const int sx1 = (e[u] >> 24) & 1 ? sx : sx + 1;
                        p00[u] = S0[sx];
                        p01[u] = S0[sx1];
                        p10[u] = S1[sx];
                        p11[u] = S1[sx1];
                    }
#pragma unroll
                    for (int u = 0; u < kPyrUnroll; ++u) {
                        const int x = x0 + 64 * u + lane;
                        if (x >= w) break;
                        const bool cr = (e[u] >> 24) & 1;
                        // right-border column: H = S[sx] * 2048 (a0 = 2048, a1 = 0)
                        const unsigned a0 = cr ? 2048u : (e[u] >> 10) & 4095;
                        const unsigned a1 = cr ? 0u : 2047u - ((e[u] >> 10) & 4095) + ((e[u] >> 22) & 3);
                        const unsigned h0 = __umul24(p00[u], a0) + __umul24(p01[u], a1);
                        const unsigned h1 = __umul24(p10[u], a0) + __umul24(p11[u], a1);
                        // 8U specialisation (default) or the generic fixed-point cast (A.1 switch)
                        int v;
                        if (!generic)
                            v = (int)(((__umul24(b0, h0 >> 4) >> 16) + (__umul24(b1, h1 >> 4) >> 16) + 2) >> 2);
                        else
                            v = min((int)((b0 * h0 + b1 * h1 + (1u << 21)) >> 22), 255);
                        D[x] = (uint8_t)v;
                        if (R) R[x] = (uint8_t)v;
                    }
                }
                ++y;
                // one wave: its LDS row writes precede the next level's reads in
                // program order (compiler ordering point only)
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            }
            prod[l] = y;
            if (y == y_start) break;  // nothing new at level l: deeper levels have no new source rows
            avail = y;
        }
        lds_publish(s_consumed, r + 1, lane);
    }
}

// ---------------------------------------------------------------------------
// K1a', small batches: one launch per level (level l from level l-1 in HBM /
// L2), thread = 4 consecutive output pixels of one row, the whole chip on
// every level.  The streaming kernel above runs one resizer wave per frame
// through all 7 chained levels: at one frame that is a 2.6 ms serial chain
// for 1.6 MB.  Same arithmetic, same packed column table,
// same 8U / generic switch.  Level 1 reads the caller's frames (level 0's
// plane is written later by orb_blur_fast_kernel).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void orb_resize_level_kernel(const uint8_t* __restrict__ src, size_t s_frame,
                                                               size_t s_row, int sw, int sh, uint8_t* __restrict__ dst,
                                                               size_t d_frame, int w, int h, double scy,
                                                               const uint32_t* __restrict__ T, int generic) {
    PLVI_ORB_PRIO_SET();
    const int qpr = (w + 3) >> 2;  // quads per row
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qpr * h) return;
    const int f = blockIdx.y;
    const int y = i / qpr, x0 = (i - y * qpr) * 4;
    float fy = (float)((y + 0.5) * scy - 0.5);
    int sy = (int)fy;
    sy -= (sy > fy);
    fy -= (float)sy;
    const int r0 = min(max(sy, 0), sh - 1), r1 = min(max(sy + 1, 0), sh - 1);
    const unsigned b0 = (unsigned)__builtin_rintf((1.f - fy) * 2048), b1 = (unsigned)__builtin_rintf(fy * 2048);
    const uint8_t* S0 = src + (size_t)f * s_frame + (size_t)r0 * s_row;
    const uint8_t* S1 = src + (size_t)f * s_frame + (size_t)r1 * s_row;
    uint8_t* D = dst + (size_t)f * d_frame + (size_t)y * w;
    uint32_t e[4];
    unsigned p00[4], p01[4], p10[4], p11[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = x0 + u < w ? T[x0 + u] : T[x0];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int sx = e[u] & 1023;
        const int sx1 = (e[u] >> 24) & 1 ? sx : sx + 1;
        p00[u] = S0[sx];
        p01[u] = S0[sx1];
        p10[u] = S1[sx];
        p11[u] = S1[sx1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (x0 + u >= w) break;
        const bool cr = (e[u] >> 24) & 1;
        const unsigned a0 = cr ? 2048u : (e[u] >> 10) & 4095;
        const unsigned a1 = cr ? 0u : 2047u - ((e[u] >> 10) & 4095) + ((e[u] >> 22) & 3);
        const unsigned h0 = __umul24(p00[u], a0) + __umul24(p01[u], a1);
        const unsigned h1 = __umul24(p10[u], a0) + __umul24(p11[u], a1);
        int v;
        if (!generic)
            v = (int)(((__umul24(b0, h0 >> 4) >> 16) + (__umul24(b1, h1 >> 4) >> 16) + 2) >> 2);
        else
            v = min((int)((b0 * h0 + b1 * h1 + (1u << 21)) >> 22), 255);
        D[x0 + u] = (uint8_t)v;
    }
}

// ---------------------------------------------------------------------------
// K1b: 7x7 fixed-point Gaussian blur (ORBextractor.cc:1115; A.4) and FAST
// score map (A.3) of every level in one launch.  One wave per strip of up to
// kBfCols output columns x kBfRows rows: lane L holds the four columns
// x0 - 4 + 4L .. +3 as one dword (lane 0 and the lane after the last output
// lane are the 3-px halo), rows streamed top to bottom.  Vertical pass first,
// SWAR: the 7-row window holds each row as its even / odd bytes in 16-bit
// fields (tap sums <= 255 * 256 never carry across a field), 7 v_mad_u32_u24
// per field pair; horizontal pass on those sums with v_dot2_u32_u16 and the
// neighbouring lanes' pairs (DPP wave shifts).  Exact integer sums rounded
// once, so the pass order does not change the result.  The image is read once with dword
// loads and the blur / score / level-0 planes are written with dword stores.
// The exact compass pre-test of K1 (two neighbouring compass points beyond
// T) rejects ~90 % of pixels; survivors are queued (row, column) and scored
// 64 at a time from an LDS ring of the last 32 raw rows.
// ---------------------------------------------------------------------------
// A 16-row ring and 16-bit queue entries (row modulo 256: queued rows are
// never 256 rows old), 4.6 KB of LDS and <= 64 VGPRs, so 8 waves fit a SIMD
// and the launch can share CUs with region growing.  (The per-cell NMS folded
// into this kernel was bit-exact but slower at 13 KB of LDS, DESIGN.md §4;
// r05 removed it.)
constexpr int kBfFlush = 1 ? 128 : 64;  // candidates scored per flush
// ring rows 0..5 are mirrored after row kRingRows - 1, so the 7 rows around
// any ring row are contiguous and a candidate's 17 taps are one base address
// plus immediate offsets (no per-tap wrap arithmetic)
constexpr int kRingMirror = 1 ? 6 : 0;
// source rows loaded per batch, in flight while the previous batch is
// filtered (4: 75 instead of 79 VGPRs, no faster; r06 also measured the 7-row
// window read back from the LDS ring -- 64 VGPRs, two waves beside six
// growth waves, yet the step 52.3-52.4K vs 52.6-52.8K FPS: profiles/r06/ab_combo.txt)
constexpr int kBfRB = 8;
constexpr int kBfCols = 244, kBfRowsPlain = 128, kRingRows = 16, kRingW = 256,
              kBfQCap = kBfFlush - 1 + 256 + 1;  // a row adds <= 256 candidates to < kBfFlush queued

// bound_ctrl: the lane past the wave's edge reads 0 without an `old` operand
// (update_dpp(0, ...) costs a v_mov of the zero per shift)
__device__ __forceinline__ int lane_from_left(int v) {  // lane i <- lane i-1 (wave_shr:1), lane 0 <- 0
    return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ int lane_from_right(int v) {  // lane i <- lane i+1 (wave_shl:1), lane 63 <- 0
    return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ int orb_mbcnt(unsigned long long m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {  // any alignment (gfx950 unaligned access)
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ void st_u32(uint8_t* p, uint32_t v) {
    __builtin_memcpy(p, &v, 4);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}
__device__ __forceinline__ int byte_of(uint32_t v, int j) { return (int)((v >> (8 * j)) & 255u); }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b, uint32_t c) {  // a.lo*b.lo + a.hi*b.hi + c
    return __builtin_amdgcn_udot2(as_u16x2(a), as_u16x2(b), c, false);
}

__device__ __forceinline__ int fast_S_ring(const uint8_t (*rg)[kRingW], int y, int c) {
#define RG(dy, dx) ((int)rg[(y + (dy)) & (kRingRows - 1)][c + (dx)])
    const int v = RG(0, 0);
    int d[16];
    d[0] = v - RG(3, 0);
    d[1] = v - RG(3, 1);
    d[2] = v - RG(2, 2);
    d[3] = v - RG(1, 3);
    d[4] = v - RG(0, 3);
    d[5] = v - RG(-1, 3);
    d[6] = v - RG(-2, 2);
    d[7] = v - RG(-3, 1);
    d[8] = v - RG(-3, 0);
    d[9] = v - RG(-3, -1);
    d[10] = v - RG(-2, -2);
    d[11] = v - RG(-1, -3);
    d[12] = v - RG(0, -3);
    d[13] = v - RG(1, -3);
    d[14] = v - RG(2, -2);
    d[15] = v - RG(3, -1);
#undef RG
    // max over the 16 arcs of 9 contiguous points of min(arc) (brighter) and
    // of -max(arc) (darker); arcs starting at k and k+1 share d[k+1..k+8]
    int A = -1000, Bm = 1000;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = d[(k + 1) & 15], b = a;
#pragma unroll
        for (int t = 2; t <= 8; ++t) {
            a = min(a, d[(k + t) & 15]);
            b = max(b, d[(k + t) & 15]);
        }
        A = max(A, max(min(a, d[k]), min(a, d[(k + 9) & 15])));
        Bm = min(Bm, min(max(b, d[k]), max(b, d[(k + 9) & 15])));
    }
    return max(A, -Bm);
}

// fast_S_ring for two pixels at once (a in the low, b in the high 16-bit
// field of every value: v_pk_sub/min/max_i16).  Same arcs, regrouped: for an
// even k the arcs starting at k and k+1 share inner_k = min(d[k+1..k+8]), and
// max(min(d[k], in), min(in, d[k+9])) = min(in, max(d[k], d[k+9])); the eight
// inner minima are built from pair then quad minima of odd-started runs
// (d[j..j+1], d[j..j+3]), so each sense costs 47 packed ops for two pixels.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 fast_S_ring2(const uint8_t (*rg)[kRingW], int ya, int ca, int yb, int cb) {
    const uint8_t* ra = &rg[(ya - 3) & (kRingRows - 1)][ca - 3];  // rows ya-3..ya+3 contiguous (mirror)
    const uint8_t* rb = &rg[(yb - 3) & (kRingRows - 1)][cb - 3];
#define RG2(dy, dx) \
    (s16x2){(short)ra[((dy) + 3) * kRingW + (dx) + 3], (short)rb[((dy) + 3) * kRingW + (dx) + 3]}
    const s16x2 v = RG2(0, 0);
    s16x2 d[16];
    d[0] = v - RG2(3, 0);
    d[1] = v - RG2(3, 1);
    d[2] = v - RG2(2, 2);
    d[3] = v - RG2(1, 3);
    d[4] = v - RG2(0, 3);
    d[5] = v - RG2(-1, 3);
    d[6] = v - RG2(-2, 2);
    d[7] = v - RG2(-3, 1);
    d[8] = v - RG2(-3, 0);
    d[9] = v - RG2(-3, -1);
    d[10] = v - RG2(-2, -2);
    d[11] = v - RG2(-1, -3);
    d[12] = v - RG2(0, -3);
    d[13] = v - RG2(1, -3);
    d[14] = v - RG2(2, -2);
    d[15] = v - RG2(3, -1);
#undef RG2
    // the brighter sense first, then the darker one, each with its pair and
    // quad minima built in place: one sense's 8 partial runs live at a time
    // (the r03 form kept pa / pb / qa / qb together, 16 more VGPRs at the
    // kernel's register peak)
    s16x2 A = (s16x2){-1000, -1000}, Bm = (s16x2){1000, 1000};
    {
        s16x2 qa[8];  // index i <-> odd start j = 2i + 1: min(d[j], d[j+1]), then min over d[j..j+3]
#pragma unroll
        for (int i = 0; i < 8; ++i) qa[i] = __builtin_elementwise_min(d[2 * i + 1], d[(2 * i + 2) & 15]);
        const s16x2 p0 = qa[0];
#pragma unroll
        for (int i = 0; i < 8; ++i) qa[i] = __builtin_elementwise_min(qa[i], i < 7 ? qa[i + 1] : p0);
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            const int i = k / 2;  // inner run d[k+1..k+8] = quads at k+1 and k+5
            const s16x2 ia = __builtin_elementwise_min(qa[i], qa[(i + 2) & 7]);
            A = __builtin_elementwise_max(A, __builtin_elementwise_min(ia, __builtin_elementwise_max(d[k], d[(k + 9) & 15])));
        }
    }
    {
        s16x2 qb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) qb[i] = __builtin_elementwise_max(d[2 * i + 1], d[(2 * i + 2) & 15]);
        const s16x2 p0 = qb[0];
#pragma unroll
        for (int i = 0; i < 8; ++i) qb[i] = __builtin_elementwise_max(qb[i], i < 7 ? qb[i + 1] : p0);
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            const int i = k / 2;
            const s16x2 ib = __builtin_elementwise_max(qb[i], qb[(i + 2) & 7]);
            Bm = __builtin_elementwise_min(Bm, __builtin_elementwise_max(ib, __builtin_elementwise_min(d[k], d[(k + 9) & 15])));
        }
    }
    return __builtin_elementwise_max(A, -Bm);
}

// occupancy: 6 waves/SIMD, set by the 6.4 KB of LDS per wave (79 VGPRs fit
// under that; a waves-per-EU or VGPR cap above 6 waves cannot take effect)
__global__ __launch_bounds__(64) void orb_blur_fast_kernel(const OrbLevelDev* __restrict__ lvs,
                                                           const OrbStripDev* __restrict__ strips,
                                                           const uint8_t* __restrict__ frames, size_t f_frame,
                                                           size_t f_row, uint8_t* __restrict__ pyr,
                                                           uint8_t* __restrict__ blur, uint8_t* __restrict__ score,
                                                           int k0, int k1,
                                                           int k2, int k3, int tmin, int t1, int t2, int nstrips,
                                                           int nf, int copy0) {
    if (PLVI_BF_SETPRIO) __builtin_amdgcn_s_setprio(PLVI_BF_SETPRIO);
    else PLVI_ORB_PRIO_SET();
    typedef unsigned short QT;
    __shared__ __align__(16) uint8_t ring[kRingRows + kRingMirror][kRingW];
    __shared__ QT q[kBfQCap];
    // XCD-affine mapping: blocks b and b + 8 share an XCD (and its L2), so
    // every strip of a frame goes to one XCD and the rows / columns two
    // strips share are fetched from HBM once
    const int bx = blockIdx.x, xk = bx >> 3;
    const int f = (bx & 7) + 8 * (xk / nstrips);
    if (f >= nf) return;
    const OrbStripDev sd = strips[xk % nstrips];
    const int lane = threadIdx.x;
    const OrbLevelDev& L = lvs[sd.level];
    const int w = L.w, h = L.h;
    const int ax = sd.x0 & ~3;                     // 4-aligned base of the strip's columns
    const int c0 = ax - 4 + 4 * lane;              // first of this lane's four columns
    const int xe = min(sd.x1, w);
    const bool need = lane <= (xe - ax + 3) / 4 + 1;  // output lanes and the two halo lanes
    const bool inner = need && c0 >= 0 && c0 + 4 <= w;  // all four inside the row: one dword
    unsigned omask = 0;                            // this lane's output columns
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (c0 + j >= sd.x0 && c0 + j < xe) omask |= 1u << j;
    const bool outl = omask != 0u;
    const uint8_t* src = sd.level == 0 ? frames + (size_t)f * f_frame : pyr + L.off + (size_t)f * L.plane;
    const size_t srow = sd.level == 0 ? f_row : (size_t)w;
    uint8_t* Dp = pyr + L.off + (size_t)f * L.plane;
    uint8_t* Bp = blur + L.boff + (size_t)f * L.bplane;
    uint8_t* Sp = score + L.boff + (size_t)f * L.bplane;
    const int bw = L.bpitch;
    const int T = max(tmin + 1, 1);
    const int y0 = sd.y0, y1 = sd.y1;
    unsigned fastok = 0;  // pixel j may be a FAST candidate
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (((omask >> j) & 1u) && c0 + j >= 3 && c0 + j < w - 3) fastok |= 1u << j;
    // rows r-6..r as even bytes (columns c0, c0+2) and odd bytes (c0+1, c0+3) in 16-bit fields
    uint32_t pe[7] = {0, 0, 0, 0, 0, 0, 0}, po[7] = {0, 0, 0, 0, 0, 0, 0};
    const uint32_t kt[7] = {(uint32_t)k0, (uint32_t)k1, (uint32_t)k2, (uint32_t)k3,
                            (uint32_t)k2, (uint32_t)k1, (uint32_t)k0};
    auto pk = [](int lo, int hi) { return (uint32_t)lo | (uint32_t)hi << 16; };
    int nq = 0;      // queued candidates (wave-uniform)
    int oldest = 0;  // row of the oldest queued candidate
    int ynew = 0;    // row of the newest queued candidate (queue rows are stored modulo 256)
    auto ent = [&](unsigned e, int yref, int& yy, int& rc) {  // queue entry -> (row, strip column)
        yy = yref - (int)((((unsigned)yref & 255u) - (e >> 8)) & 255u);
        rc = (int)(e & 255u);
    };
    auto flush = [&](int n, int ycur) {  // score the first n (<= kBfFlush) queued candidates (ycur: newest queued row)
        // one wave per block: wave-scope ordering only (no store drain).  The
        // candidate bytes below land after this wave's earlier zero stores of
        // the same pixels: a wavefront observes its own memory operations in
        // program order (wavefront-scope acquire/release needs no waits).
        wave_sync();
        int sva = 0, svb = 0;
        const bool hasb = lane + 64 < n;
        if (lane < n) {
            int ya, ca, yb, cb;
            ent(q[lane], ycur, ya, ca);
            ent(q[hasb ? lane + 64 : lane], ycur, yb, cb);
            const s16x2 sv2 = fast_S_ring2(ring, ya, ca, yb, cb);
            sva = (int)sv2.x;
            svb = (int)sv2.y;
            Sp[(size_t)ya * bw + (ax - 4 + ca)] = (uint8_t)(sva >= T ? sva - 1 : 0);
            if (hasb) Sp[(size_t)yb * bw + (ax - 4 + cb)] = (uint8_t)(svb >= T ? svb - 1 : 0);
        }
        wave_sync();
        const int rest = nq - n;
        constexpr int kMove = (kBfQCap - kBfFlush + 63) / 64;  // rest < kBfQCap - kBfFlush + 1 entries
        QT t[kMove];
#pragma unroll
        for (int k = 0; k < kMove; ++k) t[k] = lane + 64 * k < rest ? q[n + lane + 64 * k] : (QT)0;
        wave_sync();
#pragma unroll
        for (int k = 0; k < kMove; ++k)
            if (lane + 64 * k < rest) q[lane + 64 * k] = t[k];
        nq = rest;
        wave_sync();
        oldest = rest > 0 ? ycur - (int)((((unsigned)ycur & 255u) - ((unsigned)q[0] >> 8)) & 255u) : 0;
    };
    // rows rb..rb+kBfRB-1 of the source (reflected), four columns per lane
    auto load_rows = [&](int rb, uint32_t* pv) {
#pragma unroll
        for (int k = 0; k < kBfRB; ++k) {
            const int r = rb + k;
            pv[k] = (inner && r < y1 + 3) ? ld_u32(src + (size_t)reflect1(r, h) * srow + c0) : 0u;
        }
        if (need && !inner) {  // image-edge lanes: reflected columns byte by byte
#pragma unroll
            for (int k = 0; k < kBfRB; ++k) {
                const int r = rb + k;
                if (r < y1 + 3) {
                    const uint8_t* rp = src + (size_t)reflect1(r, h) * srow;
#pragma unroll
                    for (int j = 0; j < 4; ++j) pv[k] |= (uint32_t)rp[reflect1(c0 + j, w)] << (8 * j);
                }
            }
        }
    };
    uint32_t pv[kBfRB];
    load_rows(y0 - 3, pv);
    for (int rb = y0 - 3; rb < y1 + 3; rb += kBfRB) {
        // writing rows rb..rb+kBfRB-1 replaces rows rb-kRingRows..rb-kRingRows+kBfRB-1
        // of the ring; a queued row yy needs rows yy-3..yy+3.  (The score ring
        // zeroes output rows up to rb+4, i.e. rows <= rb+4-kSRows: after this
        // every queued or NMS-pending row is >= rb-6.)
        if (nq > 0 && oldest - 3 < rb - (kRingRows - kBfRB)) flush(nq, ynew);
#pragma unroll
        for (int k = 0; k < kBfRB; ++k) {
            const int rr = (rb + k) & (kRingRows - 1);
            *reinterpret_cast<uint32_t*>(&ring[rr][4 * lane]) = pv[k];
            if (rr < kRingMirror) *reinterpret_cast<uint32_t*>(&ring[rr + kRingRows][4 * lane]) = pv[k];
        }
        // next batch in flight while this one is filtered
        if (rb + kBfRB < y1 + 3) load_rows(rb + kBfRB, pv);
#pragma unroll 1
        for (int k = 0; k < kBfRB; ++k) {
            const int r = rb + k;
            if (r >= y1 + 3) break;
            const uint32_t V = *reinterpret_cast<const uint32_t*>(&ring[r & (kRingRows - 1)][4 * lane]);
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) {
                pe[rr] = pe[rr + 1];
                po[rr] = po[rr + 1];
            }
            pe[6] = V & 0x00ff00ffu;
            po[6] = (V >> 8) & 0x00ff00ffu;
            const int y = r - 3;
            if (y < y0) continue;
            // ---- output row y: rows y-3..y+3 are pe/po[0..6]
            uint32_t E = 0, O = 0;  // vertical sums: E = (c0, c0+2), O = (c0+1, c0+3)
#pragma unroll
            for (int t = 0; t < 7; ++t) {  // fields < 2^24: v_mad_u32_u24
                E += __umul24(kt[t], pe[t]);
                O += __umul24(kt[t], po[t]);
            }
            const uint32_t pe0 = pe[0], po0 = po[0], pe3 = pe[3], po3 = po[3], pe6 = pe[6], po6 = po[6];
            const uint32_t El = (uint32_t)lane_from_left((int)E), Ol = (uint32_t)lane_from_left((int)O);
            const uint32_t Er = (uint32_t)lane_from_right((int)E), Or = (uint32_t)lane_from_right((int)O);
            // El = (c0-4, c0-2), Ol = (c0-3, c0-1), Er = (c0+4, c0+6), Or = (c0+5, c0+7)
            const unsigned h0 = udot2(Ol, pk(k0, k2), udot2(E, pk(k3, k1), udot2(O, pk(k2, k0), udot2(El, pk(0, k1), 0u))));
            const unsigned h1 = udot2(El, pk(0, k0), udot2(Ol, pk(0, k1), udot2(E, pk(k2, k2),
                                udot2(O, pk(k3, k1), udot2(Er, pk(k0, 0), 0u)))));
            const unsigned h2 = udot2(Ol, pk(0, k0), udot2(E, pk(k1, k3), udot2(O, pk(k2, k2),
                                udot2(Er, pk(k1, 0), udot2(Or, pk(k0, 0), 0u)))));
            const unsigned h3 = udot2(E, pk(k0, k2), udot2(O, pk(k1, k3), udot2(Er, pk(k2, k0), udot2(Or, pk(k1, 0), 0u))));
            const uint32_t Bv = min((h0 + 32768u) >> 16, 255u) | min((h1 + 32768u) >> 16, 255u) << 8 |
                                min((h2 + 32768u) >> 16, 255u) << 16 | min((h3 + 32768u) >> 16, 255u) << 24;
            const uint32_t cvw = pe3 | po3 << 8;
            const uint32_t L3 = __builtin_amdgcn_alignbyte(cvw, (uint32_t)lane_from_left((int)cvw), 1);   // column c-3
            const uint32_t R3 = __builtin_amdgcn_alignbyte((uint32_t)lane_from_right((int)cvw), cvw, 3);  // column c+3
            // compass pre-test on 16-bit fields (even pixels 0/2, odd pixels 1/3):
            // brighter-by-T / darker-by-T at two cyclically adjacent compass points
            // (0 = row+3, 4 = col+3, 8 = row-3, 12 = col-3)
            const uint32_t ce[2] = {pe3, po3};
            const uint32_t p0[2] = {pe6, po6}, p8[2] = {pe0, po0};
            const uint32_t p4[2] = {R3 & 0x00ff00ffu, (R3 >> 8) & 0x00ff00ffu};
            const uint32_t p12[2] = {L3 & 0x00ff00ffu, (L3 >> 8) & 0x00ff00ffu};
            unsigned candm = 0;  // bit j: pixel j passes the pre-test
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const u16x2 c = as_u16x2(ce[e]);
                const u16x2 q0 = as_u16x2(p0[e]), q4 = as_u16x2(p4[e]), q8 = as_u16x2(p8[e]), q12 = as_u16x2(p12[e]);
                // the 4 compass points form a cycle whose adjacent pairs are {0,8} x
                // {4,12}: max over pairs of min(x, y) = min(max(x0, x8), max(x4, x12)),
                // and max(c -sat q0, c -sat q8) = c -sat min(q0, q8)
                const u16x2 n08 = __builtin_elementwise_min(q0, q8), n412 = __builtin_elementwise_min(q4, q12);
                const u16x2 x08 = __builtin_elementwise_max(q0, q8), x412 = __builtin_elementwise_max(q4, q12);
                const u16x2 mb = __builtin_elementwise_min(__builtin_elementwise_sub_sat(c, n08),
                                                           __builtin_elementwise_sub_sat(c, n412));
                const u16x2 md = __builtin_elementwise_min(__builtin_elementwise_sub_sat(x08, c),
                                                           __builtin_elementwise_sub_sat(x412, c));
                const uint32_t m = as_u32(__builtin_elementwise_max(mb, md));
                candm |= ((m & 0xffffu) >= (unsigned)T ? 1u : 0u) << e;
                candm |= ((m >> 16) >= (unsigned)T ? 4u : 0u) << e;
            }
            if (!(y >= 3 && y < h - 3)) candm = 0;
            candm &= fastok;
            if (outl) {
                const uint32_t o = (uint32_t)(y * w + c0), ob = (uint32_t)(y * bw + c0);
                if (omask == 15u) {
                    if (sd.level == 0 && copy0) st_u32(Dp + o, cvw);
                    st_u32(Bp + ob, Bv);
                    st_u32(Sp + ob, 0u);  // candidates / survivors are overwritten later (wave-ordered)
                } else {
                    for (int j = 0; j < 4; ++j)
                        if ((omask >> j) & 1u) {
                            if (sd.level == 0 && copy0) Dp[o + j] = (uint8_t)byte_of(cvw, j);
                            Bp[ob + j] = (uint8_t)byte_of(Bv, j);
                            Sp[ob + j] = 0;
                        }
                }
            }
            const int nq0 = nq;
            {
                // lane-major queue order: the lane's candidate count (0..4) as three
                // ballot bit planes gives every lane its exclusive prefix with mbcnt
                const unsigned cnt = (unsigned)__popc(candm);
                const unsigned long long B0 = __ballot(cnt & 1u), B1 = __ballot(cnt & 2u), B2 = __ballot(cnt & 4u);
                if ((B0 | B1 | B2) != 0ull) {
                    const int pre = nq + orb_mbcnt(B0) + 2 * orb_mbcnt(B1) + 4 * orb_mbcnt(B2);
                    const unsigned base = ((unsigned)y & 255u) << 8 | (unsigned)(4 * lane);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if ((candm >> j) & 1u) q[pre + __popc(candm & ((1u << j) - 1u))] = (QT)(base | (unsigned)j);
                    nq += __popcll(B0) + 2 * __popcll(B1) + 4 * __popcll(B2);
                }
            }
            if (nq0 == 0 && nq > 0) oldest = y;
            if (nq > nq0) ynew = y;
            while (nq >= kBfFlush) flush(kBfFlush, ynew);
        }
    }
    while (nq > 0) flush(min(nq, kBfFlush), ynew);
}

// ---------------------------------------------------------------------------
// K2: per-cell FAST non-max suppression with the reference's threshold
// fallback (ORBextractor.cc:808-829): survivors at iniThFAST; if none in the
// cell, survivors at minThFAST.  NMS is cell-local: neighbours outside the
// cell's detection window count as 0 (cv::FAST on the cell ROI), a
// neighbour below the threshold counts as 0, and a survivor is strictly
// greater than all 8 (A.3).
// One wave per (cell, frame), lane = window column (windows are < 64 wide),
// each row's 8 neighbours from the rows above / below and DPP lane shifts.
// Survivors are appended to the (frame, level) candidate list -- one 32-bit
// entry (x, y relative to the octree region, response) each, a block of the
// list reserved per cell with one atomic (r06: the list replaces the
// candidate plane, its summed-area table and the per-node plane scans; the
// consumers, node counts and per-node maxima, do not depend on list order).
// ---------------------------------------------------------------------------
// rows loaded per round trip, the next chunk prefetched while one is swept
// (r06: a whole 40-row window per round trip, 61 VGPRs, made the step 4 %
// slower, profiles/r06/ab_nms_sat.txt)
constexpr int kNmsRows = 8;
// the (frame, level) candidate counters, one per 128-byte line: the NMS waves
// of a level (~300 at level 0) all add to theirs, and packed counters put two
// frames' levels on one line, whose atomics the L2 serialises
#ifndef PLVI_COUNT_PAD
#define PLVI_COUNT_PAD 32
#endif
constexpr int kOrbCountPad = PLVI_COUNT_PAD;
// a candidate: x | y << 11 | response << 21 (x < 2048, y < 1024 relative to
// the octree region)
__device__ __forceinline__ uint32_t orb_cand_pack(int x, int y, int resp) {
    return (uint32_t)x | (uint32_t)y << 11 | (uint32_t)resp << 21;
}
// its rank in the reference's candidate order (cell-row-major, raster within
// a cell): the node maximum's tie-break, recomputed where it is needed
__device__ __forceinline__ unsigned orb_cand_key(int x, int y, const OrbLevelDev& lv) {
    const unsigned ci = (unsigned)(y - 3) / (unsigned)lv.hCell, cj = (unsigned)(x - 3) / (unsigned)lv.wCell;
    return ((ci * (unsigned)lv.nCols + cj) * (unsigned)lv.rh + (unsigned)y) * (unsigned)lv.rw + (unsigned)x;
}
__device__ __forceinline__ void orb_nms_cell(const OrbCellDev c, const int f, const OrbLevelDev* __restrict__ lvs,
                                             const uint8_t* __restrict__ score, uint32_t* __restrict__ clist,
                                             int listFrame, int* __restrict__ ccount, int L, int* __restrict__ err,
                                             int t1, int t2) {
    const OrbLevelDev& Lv = lvs[c.level];
    const int ww = c.x1 - c.x0, wh = c.y1 - c.y0, w = Lv.bpitch;
    const int lane = threadIdx.x;
    const bool incol = lane < ww;
    const size_t base = Lv.boff + (size_t)f * Lv.bplane + (size_t)c.y0 * w + c.x0 + lane;
    const uint8_t* S = score + base;
    // Register streaming, no LDS: rows come straight from the score plane,
    // eight in flight (the next chunk is loaded while this one is swept), so
    // the kernel occupies no LDS next to the region-growing waves it runs
    // with; survivors' responses are re-read from the (L2-resident) plane.
    unsigned long long ka = 0, kb = 0;
    auto ld = [&](int r) -> int { return (incol && r < wh) ? (int)S[(size_t)r * w] : 0; };
    {
        // kNmsRows rows in flight, the next chunk loaded while this one is swept
        constexpr int R = kNmsRows;
        int nx[R];
#pragma unroll
        for (int k = 0; k < R; ++k) nx[k] = ld(1 + k);
        int s = ld(0);
        int hp = 0;
        int lr = max(lane_from_left(s), lane_from_right(s));
        int hc = max(s, lr);
        for (int r0 = 0; r0 < wh; r0 += R) {
            int cur[R];
#pragma unroll
            for (int k = 0; k < R; ++k) cur[k] = nx[k];
            if (r0 + R < wh) {
#pragma unroll
                for (int k = 0; k < R; ++k) nx[k] = ld(r0 + R + 1 + k);
            }
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int r = r0 + k;
                if (r < wh) {
                    const int sn = cur[k];
                    const int lrn = max(lane_from_left(sn), lane_from_right(sn));
                    const int hn = max(sn, lrn);
                    const int m = max(max(hp, hn), lr);
                    if (s > m) {
                        if (s >= t1) ka |= 1ull << r;
                        if (s >= t2) kb |= 1ull << r;
                    }
                    hp = hc;
                    hc = hn;
                    lr = lrn;
                    s = sn;
                }
            }
        }
    }
    const unsigned long long keep = __ballot(ka != 0ull) != 0ull ? ka : kb;
    // reserve the cell's block of the list: wave prefix of the per-lane counts
    const int nk = incol ? __popcll(keep) : 0;
    int pre = nk;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(pre, o);
        if (lane >= o) pre += t;
    }
    const int tot = __shfl(pre, 63);
    if (tot == 0) return;
    int b0 = 0;
    if (lane == 0) b0 = atomicAdd(ccount + ((size_t)f * L + c.level) * kOrbCountPad, tot);
    b0 = __shfl(b0, 0);
    if (lane == 0 && b0 + tot > Lv.listCap) atomicOr(err + f, 1);  // cannot happen: listCap bounds the survivors
    int pos = b0 + pre - nk;
    uint32_t* out = clist + (size_t)f * listFrame + Lv.listOff;
    const int xr = c.x0 + lane - Lv.minB, yr0 = c.y0 - Lv.minB;
    for (unsigned long long kk = keep; incol && kk; kk &= kk - 1, ++pos) {
        const int r = __ffsll((long long)kk) - 1;
        if (pos < Lv.listCap) out[pos] = orb_cand_pack(xr, yr0 + r, S[(size_t)r * w]);
    }
}

__global__ __launch_bounds__(64) void orb_cell_nms_kernel(const OrbCellDev* __restrict__ cells, int ncells,
                                                          const OrbLevelDev* __restrict__ lvs,
                                                          const uint8_t* __restrict__ score,
                                                          uint32_t* __restrict__ clist, int listFrame,
                                                          int* __restrict__ ccount, int L, int* __restrict__ err,
                                                          int t1, int t2) {
    PLVI_ORB_PRIO_SET();
    const int f = blockIdx.y;
    for (int ci = blockIdx.x; ci < ncells; ci += gridDim.x)
        orb_nms_cell(cells[ci], f, lvs, score, clist, listFrame, ccount, L, err, t1, t2);
}

// ---------------------------------------------------------------------------
// K3: ORBextractor::DistributeOctTree (ORBextractor.cc:537-761) as a list
// emulation over node rectangles, then "retain the best point in each node"
// (:739-758).  A node's key set is the set of candidates inside its
// membership rectangle, so DivideNode's vKeys copies are replaced by counts
// over the (frame, level) candidate list; the std::list order (children
// pushed to the FRONT in n1..n4 order, parent erased), the bNoMore flags,
// both termination tests and the phase-2 (size, node*) sort are reproduced
// exactly, with the canonical creation-order tie-break of SURVEY.md B.1.
// Each final node keeps its maximum-response candidate, ties to the first in
// the reference's candidate order (cell-row-major, raster within a cell: a
// key of the coordinates).  One wave per (level, frame); the list emulation
// runs in lockstep on every lane, the counts and maxima over the candidates
// with the whole wave.  Output: the level keypoints in node list order.
// ---------------------------------------------------------------------------
struct OctNodes {
    short *gx0, *gy0, *gx1, *gy1;  // geometry UL=(gx0,gy0) BR=(gx1,gy1)
    short *mx0, *my0, *mx1, *my1;  // membership rectangle (half-open)
    int *cnt, *seq;
    short *nxt, *prv, *freel;
    short *vsz, *vprev, *todo;
    int* ccnt;                     // [C][4] key counts of the four children (prefetched)
    int* beg;                      // [C] first entry of the node's range in the partitioned list
    unsigned char* nomore;
};
constexpr int kOctListLds = 1536;  // candidates of a (frame, level) staged in LDS (more: read from the list in memory)
// dynamic LDS of orb_octree_kernel: the node arrays, then the staged candidates
__host__ __device__ inline size_t orb_octree_lds_nodes(int nodeCap) { return ((size_t)nodeCap * (7 * 4 + 14 * 2 + 1) + 15) & ~(size_t)15; }
__host__ __device__ inline size_t orb_octree_lds(int nodeCap, int lcap) { return orb_octree_lds_nodes(nodeCap) + 8 * (size_t)lcap; }

__global__ __launch_bounds__(64) void orb_octree_kernel(const OrbLevelDev* __restrict__ lvs,
                                                        const uint32_t* __restrict__ clist, int listFrame,
                                                        const int* __restrict__ ccount, float4* __restrict__ lvkp,
                                                        int kpCapFrame, int* __restrict__ out_cnt, int nodeCapMax,
                                                        int L, int* __restrict__ err, int lcap) {
    PLVI_ORB_PRIO_SET();
    extern __shared__ __align__(16) unsigned char smem[];
    // grid (frames, levels): every frame's level 0 (the longest waves) is
    // dispatched first and the short high levels fill the tail (longest
    // first); consecutive blocks are consecutive frames, dealt round-robin
    // over the 8 XCDs.  The r05-r06 grid (levels, frames) with the level
    // rotated by the frame mixed the levels through the launch: ORB chain
    // 20.3 -> 18.9 ms at 3072 frames (profiles/r06/ab_octree_lpt.txt)
    const int f = blockIdx.x, l = blockIdx.y, lane = threadIdx.x;
    const OrbLevelDev& lv = lvs[l];
    const int C = nodeCapMax;
    OctNodes n;
    uint32_t* lcache;
    {
        int* ip = reinterpret_cast<int*>(smem);
        n.cnt = ip; ip += C;
        n.seq = ip; ip += C;
        n.ccnt = ip; ip += 4 * C;
        n.beg = ip; ip += C;
        short* sp = reinterpret_cast<short*>(ip);
        n.gx0 = sp; sp += C; n.gy0 = sp; sp += C; n.gx1 = sp; sp += C; n.gy1 = sp; sp += C;
        n.mx0 = sp; sp += C; n.my0 = sp; sp += C; n.mx1 = sp; sp += C; n.my1 = sp; sp += C;
        n.nxt = sp; sp += C; n.prv = sp; sp += C; n.freel = sp; sp += C;
        n.vsz = sp; sp += C; n.vprev = sp; sp += C; n.todo = sp; sp += C;
        n.nomore = reinterpret_cast<unsigned char*>(sp);
        lcache = reinterpret_cast<uint32_t*>(smem + orb_octree_lds_nodes(C));
    }
    const int RW = lv.rw, RH = lv.rh;
    // the level's candidates: in LDS when they fit (the usual case), else read from memory
    const int K = min(ccount[((size_t)f * L + l) * kOrbCountPad], lv.listCap);
    const uint32_t* G = clist + (size_t)f * listFrame + lv.listOff;
    const bool inLds = K <= lcap;
    // In LDS the candidates are kept partitioned like the reference's vKeys
    // (ORBextractor.cc:616-641 hands each child its own keys): every node owns
    // a range [beg, beg + cnt) of A, children are split off stably (T is the
    // scatter buffer), so a node's counts read only its own range.  The key
    // (candidate order) is recomputed from (x, y) where it is needed.
    uint32_t* A = lcache;
    uint32_t* T = A + lcap;
    if (inLds)
        for (int i = lane; i < K; i += 64) A[i] = G[i];
    wave_sync();
    // stable split of [b, b + m) into groups 0..ng-1 (ng <= 8) of cls(entry);
    // group counts to cnt[] (LDS); group q starts at b + cnt[0] + ... + cnt[q-1]
    auto partition = [&](int b, int m, int ng, auto cls, int* cnt) {
        int c[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) c[q] = 0;
        for (int j = 0; j < m; j += 64) {
            const int g = j + lane < m ? cls(A[b + j + lane]) : -1;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q < ng) c[q] += __popcll(__ballot(g == q));
        }
        int o[8], acc = b;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            o[q] = acc;
            if (q < ng) { cnt[q] = c[q]; acc += c[q]; }
        }
        for (int j = 0; j < m; j += 64) {
            const uint32_t e = j + lane < m ? A[b + j + lane] : 0u;
            const int g = j + lane < m ? cls(e) : -1;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q < ng) {
                    const unsigned long long bal = __ballot(g == q);
                    if (g == q) T[o[q] + orb_mbcnt(bal)] = e;
                    o[q] += __popcll(bal);
                }
        }
        wave_sync();
        for (int j = b + lane; j < acc; j += 64) A[j] = T[j];
        wave_sync();
    };
    // candidates in [x0, x1) x [y0, y1), with the whole wave
    auto count = [&](int x0, int y0, int x1, int y1) -> int {
        int c = 0;
        for (int b = 0; b < K; b += 64) {
            const int i = b + lane;
            const uint32_t e = i < K ? G[i] : 0xFFFFFFFFu;
            const int x = (int)(e & 2047u), y = (int)((e >> 11) & 1023u);
            c += __popcll(__ballot(i < K && x >= x0 && x < x1 && y >= y0 && y < y1));
        }
        return c;
    };
    // the four children's counts of nodes ids[0..k): every candidate chunk
    // against each node, one ballot per child
    auto prefetch = [&](const short* ids, int k) {
        wave_sync();  // one wave per block
        for (int t = 0; t < k; ++t) {
            const int p = ids[t];
            const int x0 = n.gx0[p], y0 = n.gy0[p], x1 = n.gx1[p], y1 = n.gy1[p];
            const int midX = x0 + (int)ceilf((float)(x1 - x0) / 2), midY = y0 + (int)ceilf((float)(y1 - y0) / 2);
            if (inLds) {
                // the node's range holds exactly its members: quadrant = (x >= midX) + 2 (y >= midY)
                partition(n.beg[p], n.cnt[p], 4, [&](uint32_t e) {
                    return (int)((e & 2047u) >= (unsigned)midX) + 2 * (int)(((e >> 11) & 1023u) >= (unsigned)midY);
                }, n.ccnt + 4 * p);
                continue;
            }
            const int mx0 = n.mx0[p], my0 = n.my0[p], mx1 = n.mx1[p], my1 = n.my1[p];
            const int xa = min(mx1, midX), xb = max(mx0, midX), ya = min(my1, midY), yb = max(my0, midY);
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
            for (int b = 0; b < K; b += 64) {
                const int i = b + lane;
                const uint32_t e = i < K ? G[i] : 0xFFFFFFFFu;
                const int x = (int)(e & 2047u), y = (int)((e >> 11) & 1023u);
                const bool in = i < K && x >= mx0 && x < mx1 && y >= my0 && y < my1;
                const bool left = x < xa, right = x >= xb, top = y < ya, bottom = y >= yb;
                c0 += __popcll(__ballot(in && left && top));
                c1 += __popcll(__ballot(in && right && top));
                c2 += __popcll(__ballot(in && left && bottom));
                c3 += __popcll(__ballot(in && right && bottom));
            }
            n.ccnt[4 * p + 0] = c0;
            n.ccnt[4 * p + 1] = c1;
            n.ccnt[4 * p + 2] = c2;
            n.ccnt[4 * p + 3] = c3;
        }
        wave_sync();
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
    // Partitioned: the roots' counts are staged in ccnt (free until the first
    // prefetch).
    if (inLds)
        partition(0, K, lv.nIni, [&](uint32_t e) {
            const int x = (int)(e & 2047u);
            int g = -1;
#pragma unroll
            for (int q = 0; q < kOrbMaxRoots; ++q)
                if (q < lv.nIni && x >= lv.rootB[q] && x < lv.rootB[q + 1]) g = q;
            return g;
        }, n.ccnt);
    int rb = 0;
    for (int i = 0; i < lv.nIni; ++i) {
        const int c = inLds ? n.ccnt[i] : count(lv.rootB[i], 0, lv.rootB[i + 1], RH);
        const int cb = rb;
        rb += c;
        if (c == 0) continue;
        const int k = alloc();
        if (k < 0) break;
        n.gx0[k] = (short)lv.rootGx[i]; n.gy0[k] = 0; n.gx1[k] = (short)lv.rootGx[i + 1]; n.gy1[k] = (short)RH;
        n.mx0[k] = (short)lv.rootB[i]; n.my0[k] = 0; n.mx1[k] = (short)lv.rootB[i + 1]; n.my1[k] = (short)RH;
        n.cnt[k] = c; n.seq[k] = seqc++; n.nomore[k] = (c == 1); n.beg[k] = cb;
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
        int cc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) cc[q] = n.ccnt[4 * p + q];
        int cb = n.beg[p];  // the children's ranges follow each other in quadrant order
        for (int q = 0; q < 4; ++q) {
            int cx0, cy0, cx1, cy1, bx0, by0, bx1, by1;
            if (q == 0) { cx0 = x0; cy0 = y0; cx1 = midX; cy1 = midY; bx0 = mx0; by0 = my0; bx1 = min(mx1, midX); by1 = min(my1, midY); }
            else if (q == 1) { cx0 = midX; cy0 = y0; cx1 = x1; cy1 = midY; bx0 = max(mx0, midX); by0 = my0; bx1 = mx1; by1 = min(my1, midY); }
            else if (q == 2) { cx0 = x0; cy0 = midY; cx1 = midX; cy1 = y1; bx0 = mx0; by0 = max(my0, midY); bx1 = min(mx1, midX); by1 = my1; }
            else { cx0 = midX; cy0 = midY; cx1 = x1; cy1 = y1; bx0 = max(mx0, midX); by0 = max(my0, midY); bx1 = mx1; by1 = my1; }
            const int c = cc[q];
            cb += c;
            if (c == 0) continue;
            const int k = alloc();
            if (k < 0) return;
            n.gx0[k] = (short)cx0; n.gy0[k] = (short)cy0; n.gx1[k] = (short)cx1; n.gy1[k] = (short)cy1;
            n.mx0[k] = (short)bx0; n.my0[k] = (short)by0; n.mx1[k] = (short)bx1; n.my1[k] = (short)by1;
            n.cnt[k] = c; n.seq[k] = seqc++; n.nomore[k] = (c == 1); n.beg[k] = cb - c;
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
        // the nodes this pass splits: every node without bNoMore, in list order
        int nt = 0;
        for (int it = head; it >= 0; it = n.nxt[it])
            if (!n.nomore[it]) n.todo[nt++] = (short)it;
        prefetch(n.todo, nt);
        for (int t = 0; t < nt && !overflow; ++t) {
            const int it = n.todo[t];
            split(it, &nToExpand);
            if (overflow) break;
            unlink(it);
        }
        if (overflow) break;
        if (size >= N || size == prevSize) {
            finish = true;
        } else if (size + nToExpand * 3 > N) {
            while (!finish && !overflow) {
                prevSize = size;
                const int np = nv;
                nv = 0;
                // sort(vPrevSizeAndPointerToNode) by (size, node) ascending, the
                // node order being creation order (seq, unique): a rank sort with
                // the whole wave -- lane i ranks entries i, i+64, ... against all
                // np keys staged in ccnt (free until this phase's prefetch) -- into
                // vprev.  (The r01-r05 lane-lockstep insertion sort was a chain of
                // ~np^2/4 dependent LDS round trips: ~5.6K steps at level 0.)
                wave_sync();
                for (int i = lane; i < np; i += 64) {
                    const int v = n.vsz[i];
                    n.ccnt[i] = n.cnt[v];
                    n.ccnt[C + i] = n.seq[v];
                }
                wave_sync();
                for (int b0 = 0; b0 < np; b0 += 256) {
                    int kh[4], kl[4], rk[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int i = b0 + lane + 64 * k;
                        kh[k] = i < np ? n.ccnt[i] : 0x7fffffff;
                        kl[k] = i < np ? n.ccnt[C + i] : 0x7fffffff;
                    }
                    for (int j = 0; j < np; ++j) {
                        const int hj = n.ccnt[j], lj = n.ccnt[C + j];
#pragma unroll
                        for (int k = 0; k < 4; ++k) rk[k] += (hj < kh[k] || (hj == kh[k] && lj < kl[k])) ? 1 : 0;
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int i = b0 + lane + 64 * k;
                        if (i < np) n.vprev[rk[k]] = n.vsz[i];
                    }
                }
                wave_sync();
                prefetch(n.vprev, np);
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
    // "Retain the best point in each node" (ORBextractor.cc:739-758): lane
    // j keeps the maximum of (response, first in candidate order) over nodes
    // j, j + 64, ... of the list; every candidate is read once per 64 nodes
    int cntOut = 0;
    if (!overflow) {
        for (int it = head; it >= 0 && cntOut < lv.nodeCap; it = n.nxt[it]) n.todo[cntOut++] = (short)it;
        if (size > lv.nodeCap) overflow = true;
    }
    wave_sync();
    if (!overflow && inLds) {
        // lane j: node j's own range (the key -- candidate order -- from (x, y))
        float4* out = lvkp + (size_t)f * kpCapFrame + lv.kpOff;
        for (int j = lane; j < cntOut; j += 64) {
            const int p = n.todo[j];
            const int b = n.beg[p], m = n.cnt[p];
            unsigned long long best = 0;
            for (int i = b; i < b + m; ++i) {
                const uint32_t e = A[i];
                const int x = (int)(e & 2047u), y = (int)((e >> 11) & 1023u), resp = (int)(e >> 21);
                const unsigned key = orb_cand_key(x, y, lv);
                const unsigned long long pk = ((unsigned long long)resp << 32) | (0xFFFFFFFFu - key);
                if (pk > best) best = pk;
            }
            const unsigned key = 0xFFFFFFFFu - (unsigned)(best & 0xFFFFFFFFu);
            const unsigned xx = key % (unsigned)RW;
            const unsigned yy = (key / (unsigned)RW) % (unsigned)RH;
            out[j] = make_float4((float)(xx + lv.minB), (float)(yy + lv.minB), (float)(best >> 32), 0.f);
        }
    } else if (!overflow) {
        float4* out = lvkp + (size_t)f * kpCapFrame + lv.kpOff;
        for (int j0 = 0; j0 < cntOut; j0 += 4 * 64) {
            // nodes j0 + lane + 64 k, k < 4, in registers; one pass over the candidates
            int bx0[4], by0[4], bx1[4], by1[4];
            unsigned long long best[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + lane + 64 * k;
                bx0[k] = by0[k] = bx1[k] = by1[k] = 0;
                best[k] = 0;
                if (j < cntOut) {
                    const int p = n.todo[j];
                    bx0[k] = n.mx0[p]; by0[k] = n.my0[p]; bx1[k] = n.mx1[p]; by1[k] = n.my1[p];
                }
            }
            for (int i = 0; i < K; ++i) {
                const uint32_t e = G[i];
                const int x = (int)(e & 2047u), y = (int)((e >> 11) & 1023u), resp = (int)(e >> 21);
                const unsigned long long pk = ((unsigned long long)resp << 32) | (0xFFFFFFFFu - orb_cand_key(x, y, lv));
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x >= bx0[k] && x < bx1[k] && y >= by0[k] && y < by1[k] && pk > best[k]) best[k] = pk;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = j0 + lane + 64 * k;
                if (j < cntOut) {
                    const unsigned key = 0xFFFFFFFFu - (unsigned)(best[k] & 0xFFFFFFFFu);
                    const unsigned xx = key % (unsigned)RW;
                    const unsigned yy = (key / (unsigned)RW) % (unsigned)RH;
                    out[j] = make_float4((float)(xx + lv.minB), (float)(yy + lv.minB), (float)(best[k] >> 32), 0.f);
                }
            }
        }
    }
    if (lane == 0) {
        out_cnt[(size_t)f * L + l] = overflow ? 0 : cntOut;
        if (overflow) atomicOr(err + f, 1);
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
//  * both neighbourhoods are staged in LDS with unaligned dword loads issued
//    together (one memory round trip): the level image's 31x32 disc box for
//    IC_Angle and the blurred level's 37x37 box for rBRIEF (rotated pattern
//    offsets are within +-18);
//  * IC_Angle moments: lanes 0..30 / 32..62 take the disc columns u=-15..15
//    of rows v = 0..7 / 8..15; integer sums, so any order is exact;
//  * rBRIEF: the pattern is held in registers (loaded once per wave); lane l
//    evaluates tests l, l+64, l+128, l+192 and one ballot per 64 tests yields
//    8 descriptor bytes directly (test j = byte j/8, bit j%8).
constexpr int kDescR = 18, kDescP = 2 * kDescR + 1, kDescPitch = 40;
constexpr int kAngR = 15, kAngRows = 2 * kAngR + 1, kAngPitch = 32;

#ifndef PLVI_DESC_WPE
#define PLVI_DESC_WPE 8
#endif
#ifndef PLVI_DESC_UNROLL
#define PLVI_DESC_UNROLL 1  // rBRIEF loop unroll (4: more VGPRs for no gain once the staging is lean)
#endif
#define PLVI_PRAGMA(x) _Pragma(#x)
#define PLVI_UNROLL(n) PLVI_PRAGMA(unroll n)
__device__ __forceinline__ float uniform_f(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
// Register budget (r06): <= 64 VGPRs, so two describe waves fit a SIMD beside
// six 64-VGPR region-growing waves of the other batch (one at 92 VGPRs, which
// stretched every in-schedule launch to ~50 ms for 4 ms of work).  The
// keypoint record is read once per wave into SGPRs, both boxes are addressed
// from scalar bases with one 32-bit lane offset per load (no 64-bit VGPR
// address pairs), and the LDS layouts are linear in the lane index (the IC box
// is 8 dwords a row, the blur box 10), so every staging store is one base
// register plus an immediate offset.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PLVI_DESC_WPE))) void orb_describe_kernel(const OrbLevelDev* __restrict__ lvs, int L,
                                                           const uint8_t* __restrict__ pyr,
                                                           const uint8_t* __restrict__ blur,
                                                           const int* __restrict__ rect_cnt,
                                                           float4* __restrict__ lvkp, uint8_t* __restrict__ lvdesc,
                                                           int kpCapFrame, const uint8_t* __restrict__ frames0,
                                                           size_t f_frame, size_t f_row) {
    PLVI_ORB_PRIO_SET();
    __shared__ __align__(16) uint8_t patch[4][kDescP * kDescPitch];
    __shared__ __align__(16) uint8_t ipatch[4][kAngRows * kAngPitch];
    const int f = blockIdx.y;
    // the wave index read uniformly: the slot walk, the level record and the
    // box bases derived from it stay scalar (SGPR addresses, not 64-bit VGPR pairs)
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    uint8_t* P = patch[wv];
    uint8_t* IP = ipatch[wv];
    const int half = lane >> 5, u = (lane & 31) - 15;
    // this lane's four tests (x0, y0, x1, y1) of tests lane + 64k, packed as
    // four signed bytes per test (4 VGPRs instead of 16: one more wave per SIMD)
    uint32_t pat[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = lane + 64 * k;
        pat[k] = (uint32_t)(uint8_t)c_pattern[4 * j] | (uint32_t)(uint8_t)c_pattern[4 * j + 1] << 8 |
                 (uint32_t)(uint8_t)c_pattern[4 * j + 2] << 16 | (uint32_t)(uint8_t)c_pattern[4 * j + 3] << 24;
    }
    // the next keypoint's coordinates are loaded one slot ahead, so each
    // keypoint costs one dependent global round trip (its boxes), not two
    const int stride = gridDim.x * 4;
    const int* cnt = rect_cnt + (size_t)f * L;
    auto next_slot = [&](int s, int& lvl) {
        for (; s < kpCapFrame; s += stride) {
            lvl = 0;
            while (lvl + 1 < L && s >= lvs[lvl + 1].kpOff) ++lvl;
            if (s - lvs[lvl].kpOff < cnt[lvl]) return s;
        }
        return kpCapFrame;
    };
    auto load_kp = [&](int s) {  // the wave's keypoint record, in SGPRs
        const float4 v = lvkp[(size_t)f * kpCapFrame + s];
        return make_float4(uniform_f(v.x), uniform_f(v.y), uniform_f(v.z), uniform_f(v.w));
    };
    int lnext = 0;
    int snext = next_slot(blockIdx.x * 4 + wv, lnext);
    float4 kpn = snext < kpCapFrame ? load_kp(snext) : make_float4(0.f, 0.f, 0.f, 0.f);
    while (snext < kpCapFrame) {
        const int slot = snext, l = lnext;
        float4 kp = kpn;
        snext = next_slot(slot + stride, lnext);
        if (snext < kpCapFrame) kpn = load_kp(snext);
        const OrbLevelDev& lv = lvs[l];
        const int cx = (int)kp.x, cy = (int)kp.y;  // integer-valued level coords (>= 19 from every border)
        // level 0's image is the caller's frame unless the pyramid holds a copy
        // (frames0 != null: the batch's rows are not packed, or PLVI_ORB_L0_COPY)
        const bool view0 = l == 0 && frames0;
        const int W = view0 ? (int)f_row : lv.w, BW = lv.bpitch;
        // ---- stage both boxes: dword loads first, then LDS writes
        const uint8_t* I0 = (view0 ? frames0 + (size_t)f * f_frame : pyr + lv.off + (size_t)f * lv.plane) +
                            (size_t)(cy - kAngR) * W + (cx - kAngR);
        const uint8_t* B0 = blur + lv.boff + (size_t)f * lv.bplane + (size_t)(cy - kDescR) * BW + (cx - kDescR);
        uint32_t iv[4], bv[6];
        {
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // 31 rows x 8 dwords (columns cx-15 .. cx+16)
                const int i = lane + 64 * k;
                iv[k] = i < kAngRows * 8 ? ld_u32(I0 + (unsigned)((i >> 3) * W + 4 * (i & 7))) : 0u;
            }
        }
        {
#pragma unroll
            for (int k = 0; k < 6; ++k) {  // 37 rows x 10 dwords (columns cx-18 .. cx+21; cx+19.. unused)
                const int i = lane + 64 * k, r = i / 10;
                bv[k] = i < kDescP * 10 ? ld_u32(B0 + (unsigned)(r * BW + 4 * (i - 10 * r))) : 0u;
            }
        }
        {
            uint32_t* ip = reinterpret_cast<uint32_t*>(IP) + lane;  // dword i of the IC box = 4 i bytes
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (lane + 64 * k < kAngRows * 8) ip[64 * k] = iv[k];
            uint32_t* bp = reinterpret_cast<uint32_t*>(P) + lane;   // dword i of the blur box (pitch 10 dwords)
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (lane + 64 * k < kDescP * 10) bp[64 * k] = bv[k];
        }
        wave_sync();
        // ---- IC_Angle (ORBextractor.cc:75-102)
        float angle;
        {
        const uint8_t* center = IP + kAngR * kAngPitch + kAngR;
        int m_01 = 0, m_10 = 0;
        if (u <= 15) {
            if (half == 0) m_10 += u * center[u];
            for (int v = half ? 8 : 1; v <= (half ? 15 : 7); ++v) {
                const int d = c_umax[v];
                if (u >= -d && u <= d) {
                    const int vp = center[u + v * kAngPitch], vm = center[u - v * kAngPitch];
                    m_01 += v * (vp - vm);
                    m_10 += u * (vp + vm);
                }
            }
        }
        for (int s2 = 32; s2 > 0; s2 >>= 1) {
            m_01 += __shfl_xor(m_01, s2);
            m_10 += __shfl_xor(m_10, s2);
        }
        angle = plvi_fast_atan2((float)m_01, (float)m_10);
        if (lane == 0) {
            kp.w = angle;
            lvkp[(size_t)f * kpCapFrame + slot] = kp;
        }
        }
        // ---- rBRIEF (computeOrbDescriptor, ORBextractor.cc:106-145)
        const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
        const float ang = angle * factorPI;
        // ang in [0, 2*pi]: the branch-free glibc sincosf (exhaustively equal to
        // plvi_sinf / plvi_cosf on [0, 120), tests/native/libm_check.cpp); the
        // general form's large-argument reduction tripled the register count
        float a, b;
        plvi_sincosf_pos(ang, &b, &a);
        uint64_t* out = reinterpret_cast<uint64_t*>(lvdesc + ((size_t)f * kpCapFrame + slot) * 32);
        PLVI_UNROLL(PLVI_DESC_UNROLL)
        for (int k = 0; k < 4; ++k) {
            const float px0 = (float)(int8_t)(pat[k] & 0xffu), py0 = (float)(int8_t)((pat[k] >> 8) & 0xffu);
            const float px1 = (float)(int8_t)((pat[k] >> 16) & 0xffu), py1 = (float)(int8_t)(pat[k] >> 24);
            // GET_VALUE's x*b + y*a and x*a - y*b: the left product fused
            // (ORBextractor.cc.o, 16 vfmadd/vfmsub pairs per descriptor byte)
            const int t0 = P[(cv_round_f(rfmaf(px0, b, py0 * a)) + kDescR) * kDescPitch +
                             cv_round_f(rfmaf(px0, a, -(py0 * b))) + kDescR];
            const int t1 = P[(cv_round_f(rfmaf(px1, b, py1 * a)) + kDescR) * kDescPitch +
                             cv_round_f(rfmaf(px1, a, -(py1 * b))) + kDescR];
            const unsigned long long m = __ballot(t0 < t1);
            if (lane == 0) out[k] = m;
        }
        wave_sync();  // the next slot's staging overwrites the boxes
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
