// lines_kernels.hpp — HIP/CDNA4 kernels of the line front end:
//   LSDDetectorC (Thirdparty/line_descriptor/src/LSDDetector_custom.cpp)
//   LineSegmentDetectorImpl::flsd (src/LSD/lsd.cpp, refine = NONE)
//   BinaryDescriptor LBD (Thirdparty/line_descriptor/src/binary_descriptor_custom.cpp)
// Compiled with -ffp-contract=off (bit-exact f32/f64 sequences).
#include <hip/hip_runtime.h>

#include "lines_device.h"
#include "plvi_common.h"
#include "plvi_math.h"
#include "std_sort.h"

namespace plvi {

constexpr double kNotdef = -1024.0;
constexpr float kNotdefF = -1024.0f;
constexpr double kD2R = 3.14159265358979323846 / 180;  // DEG_TO_RADS (lsd.cpp)
constexpr double kPi = 3.14159265358979323846;
// log10(11.0) as GCC folds it (MPFR, correctly rounded) into lsd.cpp.o's
// LOG_NT (.rodata 1.0413926851582251); glibc's log10(11.0) is one ulp lower
constexpr double kLog10Of11 = 0x1.0a98b6050c56fp+0;

// ---------------------------------------------------------------------------
// LK1: LSDDetectorC::ComputePyramid level 1 = resize(level0, (w/2,h/2)).
// Exact factor 2 -> OpenCV's INTER_AREA fast path: the SIMD
// body (first floor(w/8)*8 columns) rounds (a+b+c+d+2)>>2, the scalar tail
// cvRound(sum*0.25f).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lsd_half_kernel(const uint8_t* __restrict__ src, size_t s_frame, size_t s_row,
                                                       uint8_t* __restrict__ dst, int dw, int dh, size_t d_frame) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= dw * dh) return;
    const int y = i / dw, x = i % dw;
    const uint8_t* S0 = src + (size_t)f * s_frame + (size_t)(2 * y) * s_row;
    const uint8_t* S1 = S0 + s_row;
    const int s = S0[2 * x] + S0[2 * x + 1] + S1[2 * x] + S1[2 * x + 1];
    const int simd = (dw / 8) * 8;
    int v = x < simd ? (s + 2) >> 2 : (int)__builtin_rintf((float)s * 0.25f);
    dst[(size_t)f * d_frame + (size_t)y * dw + x] = (uint8_t)min(max(v, 0), 255);
}

// ---------------------------------------------------------------------------
// LK2: LSD preparation (lsd.cpp:412-584): u8 -> f64, GaussianBlur(7x7,
// sigma = 0.6/SCALE) f64 reflect-101 (RowFilter sequential sum,
// SymmColumnFilter; lsd.cpp:455), resize x SCALE f64 INTER_LINEAR with
// float coefficients (lsd.cpp:457), ll_angle gradient / norm / fastAtan2
// (lsd.cpp:561-584); outputs per scaled pixel the angle in degrees (float,
// NOTDEF = -1024), modgrad (f64) and, for defined pixels,
// cos/sin(float(angle)) (float2).  One wave per column strip of the
// scaled image, rows streamed top to bottom: lane l holds blurred-image
// column gx0 - 3 + l.  Per source row the 7 horizontal taps come from the
// neighbouring lanes (DPP wave shifts of the byte), the 7 vertical taps from
// a register window of 7 row sums; each G row that completes a scaled row
// (yrow[2dy+1] == g) is interpolated at the lane holding xofs[dx], gathered
// to compact lane dx - X0 (bpermute) and, with the previous scaled row,
// turned into the gradient / angle / cos-sin of scaled row dy - 1.  Rows are
// prefetched 7 ahead; nothing but the wave's own registers is re-read.
// Strip table (host, LinePipeline::init): output columns [X0, X1), compact
// columns computed nc = X1 - X0 (+1: the gradient's right neighbour), all
// G columns needed within lanes 3..60.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double shfl_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)(b & 0xffffffff), src);
    const int hi = __shfl((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int dpp_from_right(int v) {  // lane i <- lane i+1 (wave_shl:1), edge lane 0
    return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ int dpp_from_left(int v) {  // lane i <- lane i-1 (wave_shr:1), edge lane 0
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ double dpp_from_right_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_from_right((int)(b & 0xffffffff)), hi = dpp_from_right((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ __launch_bounds__(64) void lsd_prep_kernel(const uint8_t* __restrict__ src, size_t s_frame, size_t s_row,
                                                       int gw, int gh, int sw, int sh, const int4* __restrict__ strips,
                                                       const int4* __restrict__ bands,
                                                       const int* __restrict__ xofs, const float* __restrict__ xa,
                                                       int xmax, const int* __restrict__ yrow,
                                                       const float* __restrict__ yb, double k0, double k1, double k2,
                                                       double k3, double rho, float* __restrict__ pix,
                                                       double* __restrict__ modgrad, float2* __restrict__ pixcs,
                                                       size_t p_frame) {
    __shared__ int hostdx[64];
    const int4 sd = strips[blockIdx.x];
    const int f = blockIdx.y;
    // row band: scaled rows [dyA, dyB) from source rows ybase0.. (the band's
    // first G row needs the 6 rows above it; earlier rows of the 7-slot
    // window are never read)
    const int4 bd = bands[blockIdx.z];
    const int dyA = bd.x, dyB = bd.y, ybase0 = bd.z;
    const int dyEnd = dyB < sh ? dyB + 1 : sh;  // scaled rows processed (one past the band: its Sc)
    const int X0 = sd.x, X1 = sd.y, gx0 = sd.z, nc = sd.w;
    const int lane = threadIdx.x;
    // compact lane t = lane takes scaled column X0 + t from lane Lt (the one
    // holding G column xofs[X0 + t]); which scaled column a lane hosts
    const int Lt = xofs[X0 + min(lane, nc - 1)] - gx0 + 3;
    hostdx[lane] = -1;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (lane < nc) hostdx[Lt] = X0 + lane;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int hdx = hostdx[lane];
    const bool interp = hdx >= 0 && hdx < xmax;
    const double a0 = interp ? (double)xa[2 * hdx] : 1.0, a1 = interp ? (double)xa[2 * hdx + 1] : 0.0;
    const uint8_t* S = src + (size_t)f * s_frame + reflect101(gx0 - 3 + lane, gw);
    const int nout = X1 - X0;
    float* P = pix + (size_t)f * p_frame + X0;
    double* M = modgrad + (size_t)f * p_frame + X0;
    float2* CS = pixcs + (size_t)f * p_frame + X0;
    const int yend = gh + 3;  // source rows -3 .. gh+2 (reflect-101)
    uint32_t pb[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) pb[k] = S[(size_t)reflect101(ybase0 + k, gh) * s_row];
    double Hw[7];
    double Gprev = 0.0, Gprevn = 0.0, Sp = 0.0, Spn = 0.0;
    int dy = dyA;
    // gradient / angle / cos-sin of scaled row y from rows y (Sp, Spn) and y + 1 (Sc, Scn)
    auto emit = [&](int y, double Sc, double Scn) {
        if (lane >= nout) return;
        const int x = X0 + lane;
        float deg = kNotdefF;
        double norm = 0.0;
        if (x < sw - 1 && y < sh - 1) {
            const double DA = Scn - Sp;
            const double BC = Spn - Sc;
            const double gx = DA + BC, gy = DA - BC;
            norm = __builtin_sqrt(rfma(gx, gx, gy * gy) / 4);  // fused in lsd.cpp.o ll_angle
            if (!(norm <= rho)) deg = plvi_fast_atan2((float)gx, (float)-gy);
        }
        const size_t o = (size_t)y * sw + lane;
        P[o] = deg;
        M[o] = norm;
        if (deg != kNotdefF) {
            float ps, pc;
            plvi_sincosf_pos((float)((double)deg * kD2R), &ps, &pc);
            CS[o] = make_float2(pc, ps);
        }
    };
    for (int ybase = ybase0; ybase < yend && dy < dyEnd; ybase += 7) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const int y = ybase + k;
            if (y >= yend || dy >= dyEnd) break;
            const int v0 = (int)pb[k];
            if (y + 7 < yend) pb[k] = S[(size_t)reflect101(y + 7, gh) * s_row];
            // RowFilter: sequential sum over columns c-3 .. c+3
            const int r1 = dpp_from_right(v0), r2 = dpp_from_right(r1), r3 = dpp_from_right(r2);
            const int l1 = dpp_from_left(v0), l2 = dpp_from_left(l1), l3 = dpp_from_left(l2);
            double s = k0 * (double)l3;
            s += k1 * (double)l2;
            s += k2 * (double)l1;
            s += k3 * (double)v0;
            s += k2 * (double)r1;
            s += k1 * (double)r2;
            s += k0 * (double)r3;
            Hw[k] = s;  // slot k = source row ybase + k
            const int g = y - 3;
            if (g < ybase0 + 3) continue;  // rows g-3 .. g+3 not all streamed yet
            // SymmColumnFilter over rows g-3 .. g+3 (slots k+1 .. k+7 mod 7)
            double G = k3 * Hw[(k + 4) % 7] + 0.0;
            G += k2 * (Hw[(k + 5) % 7] + Hw[(k + 3) % 7]);
            G += k1 * (Hw[(k + 6) % 7] + Hw[(k + 2) % 7]);
            G += k0 * (Hw[k] + Hw[(k + 1) % 7]);
            const double Gn = dpp_from_right_d(G);
            while (dy < dyEnd && yrow[2 * dy + 1] == g) {
                const bool same = yrow[2 * dy] == g;  // else g - 1
                const double G0 = same ? G : Gprev, G0n = same ? Gn : Gprevn;
                const double b0 = (double)yb[2 * dy], b1 = (double)yb[2 * dy + 1];
                double H0, H1;
                if (interp) {
                    H0 = G0 * a0 + G0n * a1;
                    H1 = G * a0 + Gn * a1;
                } else {
                    H0 = G0 * 1.0;
                    H1 = G * 1.0;
                }
                const double Sv = H0 * b0 + H1 * b1;
                const double Sc = shfl_d(Sv, Lt);
                const double Scn = dpp_from_right_d(Sc);
                if (dy > dyA) emit(dy - 1, Sc, Scn);
                Sp = Sc;
                Spn = Scn;
                ++dy;
            }
            Gprev = G;
            Gprevn = Gn;
        }
    }
    if (dyB == sh) emit(sh - 1, 0.0, 0.0);  // last row: NOTDEF (ll_angle leaves row h-1 undefined)
}

// ---------------------------------------------------------------------------
// LK3: flsd's serial core (lsd.cpp:476-533): seeds in raster order (flsd
// walks the coorlist vector, not the pseudo-ordered chain), region_grow
// (:635-686) with the exact float sumdx/sumdy/fastAtan2 update per added
// pixel, the min_reg_size test, region2rect (:688-744) + get_theta
// (:746-782) in double with the reference summation order, +0.5, /SCALE.
//
// One wave per (octave, frame).  Seeds are visited in raster order, so every
// defined pixel before the seed is already USED and a region only reaches
// rows >= seed row.  LDS therefore holds only a sliding window of R (power of
// two) rows at or below the seed row: their gradient angles and USED bits.
// Rows beyond the window are read from the angle plane and a global USED
// bitmap (L2, bypassing L1), which the window picks up when it slides.  The
// region queue lives in LDS up to QL entries and spills to global memory.
// The footprint (~37 KB at R = 16) lets four waves share a CU.
//
// Speculative exact growth: the neighbour checks of up to 7 queued points
// (63 lanes, the reference's scan order = lane order) are decided at once
// against the current region angle; the exact angle sequence implied by the
// speculated accepts is then computed (sequential float sums, parallel
// fastAtan2) and every decision is re-evaluated against the angle it would
// really see.  The consistent prefix is committed; the first inconsistent
// lane is re-decided with the exact angle in the next round.  The result is
// identical to the sequential algorithm.
// ---------------------------------------------------------------------------

struct GrowCtx {
    const float* P;   // angle plane (degrees, NOTDEF = -1024)
    unsigned* gbits;  // global USED bitmap (rows at or beyond the bits window)
    lds_u32* bits;    // LDS USED ring: RB rows x wpr words
    lds_u32* qlds;    // LDS region queue (x | y << 16), QL entries
    unsigned* qglob;  // global queue spill
    lds_f32* win;     // LDS angle ring: R rows x sw (R = 0: angles from the plane)
    int sw, sh, R, RB, wpr, wb, wbb, QL, ys;  // window bases wb (angles) / wbb (bits); ys = seed row
};

// Lanes of earlier block points (p2 < this lane's point) testing the same
// pixel: bit 9 * p2 + 3 * ddy + ddx of the block's 63 test lanes, where
// (ddx, ddy) = (nx - qx + 1, ny - qy + 1) in [0, 2]^2 for point p2 = (qx, qy).
// Both differences come from one packed 16-bit subtract, the range test from
// one packed max; bit = 9 * p2 + (3 * ny + nx + 4) - (3 * qy + qx).
typedef unsigned short plvi_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned long long dup_lanes(unsigned pv, int nb, int bp, int nx, int ny) {
    const unsigned pn1 = (unsigned)(nx + 1) | ((unsigned)(ny + 1) << 16);
    const int s = 3 * ny + nx + 4;
    unsigned long long dup = 0;
    for (int p2 = 0; p2 < nb - 1; ++p2) {
        const unsigned q2 = (unsigned)__builtin_amdgcn_readlane((int)pv, 9 * p2);
        const int t2 = 3 * (int)(q2 >> 16) + (int)(q2 & 0xffffu);
        const plvi_u16x2 d = __builtin_bit_cast(plvi_u16x2, pn1) - __builtin_bit_cast(plvi_u16x2, q2);
        const plvi_u16x2 m = __builtin_elementwise_max(d, (plvi_u16x2){2, 2});
        const bool hit = (p2 < bp) & (__builtin_bit_cast(unsigned, m) == 0x00020002u);
        const unsigned long long hm = 0ull - (unsigned long long)hit;  // a mask, not a branch
        dup |= (1ull << ((9 * p2 - t2 + s) & 63)) & hm;
    }
    return dup;
}

// lane mask of a condition (the builtin on the bool itself; the multi-wave
// growth uses it, the large-batch kernel keeps __ballot: measured either way
// within noise there, profiles/r05/grow_ab_branchless.txt)
__device__ __forceinline__ unsigned long long ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
// set bits of m below this lane (v_mbcnt_lo/hi: popcount(m & ((1 << lane) - 1)))
__device__ __forceinline__ int mbcnt64(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ unsigned gload_l2(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore_l2(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0); }

// USED test.  Rows above the seed row hold only USED or NOTDEF pixels
// (seeds are visited in raster order), so they read as USED.  The LDS read
// is unconditional (row clamped into the window); rows beyond the window
// (rare) take the global bitmap.
__device__ __forceinline__ bool used_get(const GrowCtx& g, int x, int y) {
    const bool inwin = y < g.wbb + g.RB;
    const int yy = inwin ? y : g.wbb;
    unsigned v = g.bits[(yy & (g.RB - 1)) * g.wpr + (x >> 5)];
    if (__builtin_expect(!inwin, 0)) v = gload_l2(g.gbits + (size_t)y * g.wpr + (x >> 5));
    return y < g.ys || ((v >> (x & 31)) & 1u);
}
__device__ __forceinline__ void used_set(const GrowCtx& g, int x, int y) {
    const unsigned b = 1u << (x & 31);
    if (__builtin_expect(y < g.wbb + g.RB, 1))
        __atomic_fetch_or(&g.bits[(y & (g.RB - 1)) * g.wpr + (x >> 5)], b, __ATOMIC_RELAXED);  // ds_or_b32
    else __hip_atomic_fetch_or(g.gbits + (size_t)y * g.wpr + (x >> 5), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// OR a 64-pixel chunk mask (pixels xb..xb+63 of row y, row y inside the
// window, xb a multiple of 64) into the USED bits: lanes 0 and 1 take a word each
__device__ __forceinline__ void used_set_chunk(const GrowCtx& g, int xb, int y, unsigned long long mask, int lane) {
    const unsigned w = lane == 0 ? (unsigned)mask : (unsigned)(mask >> 32);
    if (lane < 2 && w) __atomic_fetch_or(&g.bits[(y & (g.RB - 1)) * g.wpr + (xb >> 5) + lane], w, __ATOMIC_RELAXED);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}
__device__ __forceinline__ unsigned q_get(const GrowCtx& g, int i) {
    if (__builtin_expect(i < g.QL, 1)) return g.qlds[i];
    return gload_l2(g.qglob + (i - g.QL));
}
__device__ __forceinline__ void q_put(const GrowCtx& g, int i, unsigned v) {
    if (__builtin_expect(i < g.QL, 1)) g.qlds[i] = v;
    else gstore_l2(g.qglob + (i - g.QL), v);
}
__device__ __forceinline__ float deg_at(const GrowCtx& g, int x, int y) {
    if (g.R == 0) return g.P[(size_t)y * g.sw + x];
    const bool inwin = y < g.wb + g.R;
    const int yy = inwin ? y : g.wb;
    float v = g.win[(yy & (g.R - 1)) * g.sw + x];
    if (__builtin_expect(!inwin, 0)) v = g.P[(size_t)y * g.sw + x];
    return v;
}

// isAligned (lsd.cpp:1136-1152) with a = (double)deg * DEG_TO_RADS, exactly the
// value ll_angle stored in angles_data.
__device__ __forceinline__ bool is_aligned_deg(float deg, double theta, double prec) {
    // select form of the reference's branches (same operations, no divergence)
    const double a = (double)deg * kD2R;
    const double d = theta - a;
    const double n0 = d < 0 ? -d : d;
    const double d2 = n0 - (2 * kPi);
    const double n1 = d2 < 0 ? -d2 : d2;
    const double n_theta = n0 > (3 * kPi) / 2 ? n1 : n0;
    return deg != kNotdefF && n_theta <= prec;
}

// The same decision from the float degree difference T - D (theta = (double)T
// * DEG_TO_RADS, T the float fastAtan2 result the region angle comes from):
// more than 1e-3 degrees away from prec and 360 - prec the outcome is fixed
// (the 3pi/2 branch of isAligned cannot flip it there), so the double test
// runs only inside that margin (float / double rounding is < 1e-4 degrees).
__device__ __forceinline__ bool is_aligned_fast(float deg, float tdeg, float pdeg, double prec) {
    const float dd = __builtin_fabsf(tdeg - deg);
    const bool near = __builtin_fabsf(dd - pdeg) < 1e-3f || __builtin_fabsf(dd - (360.f - pdeg)) < 1e-3f;
    bool r = deg != kNotdefF && (dd <= pdeg || dd >= 360.f - pdeg);
    if (__builtin_expect(near, 0)) {
        // opaque inside the rare branch, so that its double conversions are not
        // hoisted out of the caller's loops onto the common path
        float dg = deg;
        asm volatile("" : "+v"(dg));
        r = is_aligned_deg(dg, (double)tdeg * kD2R, prec);
    }
    return r;
}

__device__ __forceinline__ double angle_diff(double a, double b) {
    double diff = a - b;
    while (diff <= -kPi) diff += (2 * kPi);
    while (diff > kPi) diff -= (2 * kPi);
    return diff < 0 ? -diff : diff;
}

// Load image rows [r0, r1) into their angle-window slots.
__device__ __forceinline__ void win_load_rows(const GrowCtx& g, int r0, int r1, int lane) {
    const int n = (r1 - r0) * g.sw;
    const float* src = g.P + (size_t)r0 * g.sw;
    int i = lane;
    for (; i + 7 * 64 < n; i += 8 * 64) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[i + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = i + u * 64, row = r0 + j / g.sw, x = j - (j / g.sw) * g.sw;
            g.win[(row & (g.R - 1)) * g.sw + x] = v[u];
        }
    }
    for (; i < n; i += 64) {
        const int row = r0 + i / g.sw, x = i % g.sw;
        g.win[(row & (g.R - 1)) * g.sw + x] = src[i];
    }
}
// Load the USED bits of rows [r0, r1) into their bits-window slots from the
// global bitmap (set while the rows were beyond the window).
__device__ __forceinline__ void bits_load_rows(const GrowCtx& g, int r0, int r1, int lane) {
    const int nw = (r1 - r0) * g.wpr;
    for (int k = lane; k < nw; k += 64) {
        const int row = r0 + k / g.wpr, w = k % g.wpr;
        g.bits[(row & (g.RB - 1)) * g.wpr + w] = gload_l2(g.gbits + (size_t)row * g.wpr + w);
    }
}

#ifndef PLVI_GROW_SETPRIO
#define PLVI_GROW_SETPRIO 3  // wave priority of the region-growing waves (s_setprio)
#endif
#ifndef PLVI_GROW_OCT1_PRIO
#define PLVI_GROW_OCT1_PRIO PLVI_GROW_SETPRIO  // priority of the octave >= 1 growth waves
#endif

// waves per SIMD the region-growing kernel is compiled for: 8 caps it at 64
// VGPRs, so its 6 resident waves per SIMD (a 3072-frame batch) leave room for
// the ORB / LBD waves of the frame schedule
#ifndef PLVI_GROW_WPE
#define PLVI_GROW_WPE 8
#endif
// waves (tasks) per workgroup of the region-growing kernel: with single-wave
// workgroups the dispatcher put 7 growth waves on 33 of the 1024 SIMDs and 5
// on 33 others at 3072 frames (every CU holds 24), and the waves on the
// 7-wave SIMDs set the launch time (max 87.9M vs 79.7M cycles on 6-wave
// SIMDs, tools/grow_stats.py); a 4-wave workgroup puts one task on each SIMD
#ifndef PLVI_GROW_WG_WAVES
#define PLVI_GROW_WG_WAVES 4
#endif
constexpr int kGrowWaves = PLVI_GROW_WG_WAVES;

// the waves of a workgroup share nothing (each has its own LDS partition):
// a wave-level barrier orders its own lanes' LDS accesses
// (the scheduling barrier keeps the code motion of the workgroup barrier it
// replaces: without it the compiler hoists loads across and spills VGPRs)
__device__ __forceinline__ void grow_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_sched_barrier(0);
}

constexpr int kGrowRB = 64, kGrowQL = 256;

template <bool STATS, bool FIXED, bool LOOP = false>
__global__ __launch_bounds__(64 * kGrowWaves, PLVI_GROW_WPE) void lsd_grow_kernel(const LineOctDev* __restrict__ octs,
                                                      const float* __restrict__ pix,
                                                      const double* __restrict__ modgrad,
                                                      const float2* __restrict__ pixcs,
                                                      unsigned* __restrict__ gbits_all, size_t gbits_frame,
                                                      unsigned* __restrict__ qspill, size_t qspill_frame,
                                                      double prec, LsdRegion* __restrict__ regs, unsigned* __restrict__ regpts,
                                                      size_t regpts_frame, int* __restrict__ nlines,
                                                      int* __restrict__ err, int R, int RB, int QL, int nOct,
                                                      int oBase, int oCount, unsigned long long* __restrict__ stats,
                                                      int nf, int ldsWave, int wpw) {
    extern __shared__ __align__(16) unsigned lds_all[];
    // latency-bound serial chain: win the SIMD arbiter against co-resident
    // throughput kernels (ORB / LBD on the other stream)
    __builtin_amdgcn_s_setprio(PLVI_GROW_SETPRIO);
    // 1-D grid, octave-major: all octave-0 tasks (4x the pixels) first, then
    // octave 1.  Blocks are dealt round-robin over the 8 XCDs, so every XCD
    // gets the same mix (a (nOct, nf) grid put every octave-0 task on the
    // even XCDs) and the heavy tasks are dispatched first.
    // this launch covers octaves oBase .. oBase + oCount - 1; task = (octave,
    // frame) in that order, wpw (<= kGrowWaves, LDS permitting) consecutive
    // tasks per workgroup; the wave index is read uniformly (readfirstlane)
    // so that everything derived from the task stays scalar
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // a grid of fewer waves than tasks (PLVI_GROW_TPW) walks them in a
    // grid-stride loop: with two tasks per wave, wave w grows octave 0 and then
    // octave 1 of frame w (no workgroup barrier below: the other waves go on)
    const int ntask = nf * oCount, tstride = LOOP ? (int)gridDim.x * wpw : ntask;
    for (int task0 = blockIdx.x * wpw + wv; task0 < ntask; task0 += tstride) {
    const int task = __builtin_amdgcn_readfirstlane(task0);
    // consecutive frames per workgroup (spreading frames over the workgroups
    // by a stride permutation was slower: 35.3 vs 33.2 ms per 3072 frames)
    const int o = oBase + task / nf, f = task - (o - oBase) * nf;
    // the octave-0 waves carry the launch (4x the pixels): PLVI_GROW_OCT1_PRIO
    // lowers the other octaves' priority below theirs
    if (PLVI_GROW_OCT1_PRIO != PLVI_GROW_SETPRIO && o > 0) __builtin_amdgcn_s_setprio(PLVI_GROW_OCT1_PRIO);
    // this wave's LDS partition, addressed as LDS (32-bit) from the start
    lds_u32* lds_w = (lds_u32*)lds_all + wv * (ldsWave >> 2);
    const LineOctDev& od = octs[o];
    const int sw = od.sw, sh = od.sh;
    const int lane = threadIdx.x & 63;
    GrowCtx g;
    if (FIXED) {  // the default windows as constants (no angle window, 64 USED rows, 256 queue entries in LDS)
        R = 0;
        RB = kGrowRB;
        QL = kGrowQL;
    }
    g.sw = sw; g.sh = sh; g.R = R; g.RB = RB; g.QL = QL;
    g.wpr = (sw + 31) >> 5;
    g.P = pix + od.soff + (size_t)f * od.splane;
    const float2* SC = pixcs + od.soff + (size_t)f * od.splane;
    LsdRegion* outR = regs + (size_t)(f * nOct + o) * kLsdRawCap;
    unsigned* outP = regpts + (size_t)(f * nOct + o) * regpts_frame;
    int npts = 0;
    g.gbits = gbits_all + (size_t)(f * nOct + o) * gbits_frame;
    g.qglob = qspill + (size_t)(f * nOct + o) * qspill_frame;
    // LDS: USED ring | queue | angle ring
    g.bits = lds_w;
    g.qlds = g.bits + RB * g.wpr;
    g.win = (lds_f32*)(g.qlds + QL);
    g.wb = 0;
    g.wbb = 0;
    g.ys = 0;
    for (int i = lane; i < sh * g.wpr; i += 64) g.gbits[i] = 0u;
    for (int i = lane; i < RB * g.wpr; i += 64) g.bits[i] = 0u;
    if (R) win_load_rows(g, 0, min(R, sh), lane);
    vm_drain();
    grow_wave_sync();
    int nout = 0;
    bool overflow = false;
    const float pdeg = (float)(prec / kD2R);  // ANG_TH in degrees
    const int min_reg = od.min_reg_size;
    const int bp = lane / 9, bk = lane % 9;  // block point / neighbour index of this lane
    const int kdx = bk % 3 - 1, kdy = bk / 3 - 1;
    const unsigned long long below = (1ull << lane) - 1ull;
    // optional cycle accounting (diagnostic): [0] total [1] block setup [2] rounds [3] rect
    // [4] seeds [5] blocks [6] rounds [7] rect points [8] commits
    unsigned long long s_setup = 0, s_round = 0, s_rect = 0, n_seed = 0, n_block = 0, n_round = 0, n_rpt = 0,
                       n_commit = 0;
    unsigned long long s_ph[4] = {0, 0, 0, 0};
    unsigned long long s_scan = 0, s_seed = 0, s_init = 0;  // seed scan, per-seed start, init
    unsigned long long n_far = 0, n_spill = 0;  // commit rounds that drained for far USED rows / queue spill
    constexpr bool do_stats = STATS;  // diagnostic variant only (keeps SGPRs free in the product kernel)
    const unsigned long long t_begin = do_stats ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long t_mark = t_begin;
    const unsigned long long t_real0 = do_stats ? __builtin_amdgcn_s_memrealtime() : 0;
    const int half = R / 2, halfb = RB / 2;
    // Seed-chunk angles, prefetched one chunk ahead from the (static) angle
    // plane: (x, y), (x-1, y), (x+1, y), (x-1, y+1), (x, y+1), (x+1, y+1)
    auto chunk_load = [&](int cy, int cxb, float* v) {
        const int x = cxb + lane, xm = max(x - 1, 0), xx = min(x, sw - 1), xp = min(x + 1, sw - 1);
        const float* r0 = g.P + (size_t)cy * sw;
        const float* r1 = r0 + sw;
        v[0] = r0[xx]; v[1] = r0[xm]; v[2] = r0[xp];
        v[3] = r1[xm]; v[4] = r1[xx]; v[5] = r1[xp];
    };
    // two chunks in flight ahead of the one being scanned (a chunk without
    // seeds takes less time than one load round trip)
    auto chunk_next = [&](int& cy, int& cxb) {
        if (cxb + 64 < sw - 1) {
            cxb += 64;
        } else {
            cxb = 0;
            ++cy;
        }
    };
    float nv[6], nv2[6];
    int py2 = 0, px2 = 0;  // chunk of nv2
    chunk_load(0, 0, nv);
    chunk_next(py2, px2);
    if (py2 < sh - 1) chunk_load(py2, px2, nv2);
    if (do_stats) s_init = __builtin_amdgcn_s_memtime() - t_begin;
    for (int y = 0; y < sh - 1; ++y) {
        // slide each window by half its height once row y is past its middle;
        // the rows leaving it are above y and never read again
        bool slid = false;
        while (R && y >= g.wb + half && g.wb + R < sh) {
            const int r0 = g.wb + R, r1 = min(sh, r0 + half);
            win_load_rows(g, r0, r1, lane);
            g.wb += r1 - r0;
            slid = true;
        }
        while (y >= g.wbb + halfb && g.wbb + RB < sh) {
            const int r0 = g.wbb + RB, r1 = min(sh, r0 + halfb);
            bits_load_rows(g, r0, r1, lane);
            g.wbb += r1 - r0;
            slid = true;
        }
        if (slid) {
            vm_drain();
            grow_wave_sync();
        }
        g.ys = y;
        for (int xb = 0; xb < sw - 1; xb += 64) {
            if (do_stats) t_mark = __builtin_amdgcn_s_memtime();
            float cv[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                cv[k] = nv[k];
                nv[k] = nv2[k];
            }
            chunk_next(py2, px2);
            if (py2 < sh - 1) chunk_load(py2, px2, nv2);
            const int x = xb + lane;
            bool cand = false, grow = false;
            if (x < sw - 1) {
                const float d0 = cv[0];
                cand = d0 != kNotdefF && !used_get(g, x, y);
                // A seed's first round tests its forward neighbours (rows above y
                // are all USED) against its own angle: when none of them is aligned
                // (a static property, whatever is USED), the region stays at size 1
                // < min_reg_size and the seed only marks itself USED.
                // neighbours (x-1,y) (x+1,y) (x-1,y+1) (x,y+1) (x+1,y+1)
                if (cand)
                    grow = (x > 0 && is_aligned_fast(cv[1], d0, pdeg, prec)) || is_aligned_fast(cv[2], d0, pdeg, prec) ||
                           (x > 0 && is_aligned_fast(cv[3], d0, pdeg, prec)) || is_aligned_fast(cv[4], d0, pdeg, prec) ||
                           is_aligned_fast(cv[5], d0, pdeg, prec);
            }
            unsigned long long m = __ballot(cand);
            if (do_stats) s_scan += __builtin_amdgcn_s_memtime() - t_mark;
            if (!m) continue;
            const unsigned long long gm = __ballot(grow);
            // USED bits of seeds that cannot grow, set before the next seed grows
            // (it must see them USED, as the reference's scan order implies)
            unsigned long long pend = m & ~gm;
            m &= gm;
            while (m) {
                const int b = __ffsll((long long)m) - 1;
                m &= m - 1;
                const int sx = xb + b;
                if (do_stats) t_mark = __builtin_amdgcn_s_memtime();
                const unsigned long long before = pend & ((1ull << b) - 1ull);
                if (before) {
                    used_set_chunk(g, xb, y, before, lane);
                    pend &= ~before;
                }
                if (used_get(g, sx, y)) continue;  // absorbed by an earlier region of this chunk
                // ---- region_grow (lsd.cpp:635-686)
                // the seed's angle is lane b's value of the scanned chunk (no reload)
                float reg_deg = readlane_f(cv[0], b);  // reg_angle = (double)reg_deg * DEG_TO_RADS
                // seed direction sumdx / sumdy: computed in the first block, while
                // its neighbourhood loads are in flight
                float sumdx = 0.f, sumdy = 0.f;
                if (lane == 0) {
                    used_set(g, sx, y);
                    g.qlds[0] = (unsigned)sx | ((unsigned)y << 16);
                }
                grow_wave_sync();
                if (do_stats) {
                    n_seed++;
                    s_seed += __builtin_amdgcn_s_memtime() - t_mark;
                }
                int reg_size = 1;
                for (int i = 0; i < reg_size;) {
                    const unsigned long long t0 = do_stats ? __builtin_amdgcn_s_memtime() : 0;
                    const int nb = min(7, reg_size - i);
                    const bool active = lane < 9 * nb;
                    // the block's queue points: one LDS read (inactive lanes read entry i),
                    // the global spill only once the queue has passed QL entries
                    unsigned pv;
                    if (i + 7 <= g.QL) {
                        const unsigned v = g.qlds[i + (active ? bp : 0)];
                        pv = active ? v : 0u;
                    } else {
                        pv = active ? q_get(g, i + bp) : 0u;
                    }
                    const int px = (int)(pv & 0xffffu), py = (int)(pv >> 16);
                    const int nx = px + kdx, ny = py + kdy;
                    const bool valid = active && nx >= 0 && nx < sw && ny >= y && ny < sh;
                    // angle and cos/sin(float(angle)) of lsd.cpp:678-679 (precomputed by
                    // lsd_prep_kernel for defined pixels) in one round trip
                    float deg = kNotdefF, cc = 0.f, ss = 0.f;
                    if (valid) {
                        const float2 cs2 = SC[(size_t)ny * sw + nx];
                        deg = deg_at(g, nx, ny);
                        cc = cs2.x;
                        ss = cs2.y;
                    }
                    if (i == 0) {
                        // sumdx = (float)cos(reg_angle), sumdy = (float)sin(reg_angle)
                        // (lsd.cpp:648-649), double libm restated (plvi_math.h), wave-uniform
                        double ds, dc;
                        plvi_sincos((double)reg_deg * kD2R, &ds, &dc);
                        sumdx = (float)dc;
                        sumdy = (float)ds;
                    }
                    // lanes of earlier block points that test the same pixel
                    unsigned long long dup = 0;
                    for (int p2 = 0; p2 < nb - 1; ++p2) {
                        const unsigned q2 = (unsigned)readlane_i((int)pv, 9 * p2);
                        const int ddx = nx - (int)(q2 & 0xffffu) + 1, ddy = ny - (int)(q2 >> 16) + 1;
                        const bool hit = p2 < bp && (unsigned)ddx <= 2u && (unsigned)ddy <= 2u;
                        // as a mask, not a branch
                        const unsigned long long hm = 0ull - (unsigned long long)hit;
                        dup |= (1ull << ((9 * p2 + ddy * 3 + ddx) & 63)) & hm;
                    }
                    unsigned long long t1 = 0;
                    if (do_stats) {
                        t1 = __builtin_amdgcn_s_memtime(); s_setup += t1 - t0; n_block++;
                    }
                    // USED is read once per block: within the block a lane's pixel
                    // only becomes USED through a commit of an earlier lane testing
                    // the same pixel (dup), tracked in Ccum
                    // (rows above the seed row are never valid lanes here)
                    const int ux = valid ? nx : 0, uy = valid ? ny : y;
                    unsigned uw = g.bits[(uy & (g.RB - 1)) * g.wpr + (ux >> 5)];
                    const bool ufar = valid && uy >= g.wbb + g.RB;
                    if (__builtin_expect(__ballot(ufar) != 0ull, 0)) {
                        if (ufar) uw = gload_l2(g.gbits + (size_t)uy * g.wpr + (ux >> 5));
                    }
                    const bool live0 = valid & (deg != kNotdefF) & (((uw >> (ux & 31)) & 1u) == 0u);
                    unsigned long long Ccum = 0;
                    int start = 0;
                    while (start < 9 * nb) {
                        unsigned long long r0t = 0;
                        if (do_stats) { n_round++; r0t = __builtin_amdgcn_s_memtime(); }
                        const unsigned long long fromStart = ~0ull << start;
                        const bool candl = lane >= start && live0 && (dup & Ccum) == 0ull;
                        const bool al = candl && is_aligned_fast(deg, reg_deg, pdeg, prec);
                        const bool acc = al && (dup & fromStart) == 0ull;
                        const unsigned long long A = __ballot(acc);
                        if (do_stats) { const unsigned long long t = __builtin_amdgcn_s_memtime(); s_ph[0] += t - r0t; r0t = t; }
                        if (!A) break;  // no commit: every remaining decision is final
                        // exact angle sequence of the speculated commits (sequential float
                        // sums); every lane keeps the sums after its cl accepted
                        // predecessors, i.e. the region angle its own test really sees
                        const int cl = mbcnt64(A);
                        float sx2 = sumdx, sy2 = sumdy, pfx = sumdx, pfy = sumdy;
                        int t = 0;
                        for (unsigned long long mm = A; mm; mm &= mm - 1) {
                            const int bl = __ffsll((long long)mm) - 1;
                            sx2 += readlane_f(cc, bl);
                            sy2 += readlane_f(ss, bl);
                            ++t;
                            if (cl == t) { pfx = sx2; pfy = sy2; }
                        }
                        const float tha = plvi_fast_atan2(pfy, pfx);
                        const float th = cl > 0 ? tha : reg_deg;
                        if (do_stats) { const unsigned long long t = __builtin_amdgcn_s_memtime(); s_ph[1] += t - r0t; r0t = t; }
                        // verify every decision against the angle it really sees
                        const bool al2 = candl && (dup & A) == 0ull && is_aligned_fast(deg, th, pdeg, prec);
                        const unsigned long long mism = __ballot(al2 != acc) & fromStart;
                        if (do_stats) { const unsigned long long t = __builtin_amdgcn_s_memtime(); s_ph[2] += t - r0t; r0t = t; }
                        // commit the consistent prefix: lanes below the first mismatch (lane
                        // 63, never a test lane, when all agree); that lane holds the sums
                        // and angle after exactly those commits
                        const int ls = mism ? __ffsll((long long)mism) - 1 : 63;
                        const unsigned long long C = A & ((1ull << ls) - 1ull);
                        const int nc = __popcll(C);
                        start = mism ? ls : 9 * nb;  // a mismatch is re-decided exactly next round
                        if (nc > 0) {
                            Ccum |= C;
                            const bool mine = (C >> lane) & 1ull;
                            const bool far = __ballot(mine && ny >= g.wbb + RB) != 0ull;
                            const bool spill = reg_size + nc > QL;
                            if (__builtin_expect(!far && !spill, 1)) {
                                // USED bit and queue entry in LDS
                                if (mine) {
                                    __atomic_fetch_or(&g.bits[(ny & (g.RB - 1)) * g.wpr + (nx >> 5)], 1u << (nx & 31),
                                                      __ATOMIC_RELAXED);
                                    g.qlds[reg_size + mbcnt64(C)] = (unsigned)nx | ((unsigned)ny << 16);
                                }
                            } else {
                                if (mine) {
                                    int sx_ = nx, sy_ = ny;  // opaque: keep the slow path's addressing here
                                    asm volatile("" : "+v"(sx_), "+v"(sy_));
                                    used_set(g, sx_, sy_);
                                    q_put(g, reg_size + mbcnt64(C), (unsigned)sx_ | ((unsigned)sy_ << 16));
                                }
                                // global USED bits / queue spill must land before they are read back
                                vm_drain();
                            }
                            if (do_stats) {
                                n_far += far;
                                n_spill += spill;
                            }
                            reg_size += nc;
                            sumdx = readlane_f(pfx, ls);
                            sumdy = readlane_f(pfy, ls);
                            reg_deg = readlane_f(th, ls);
                            if (do_stats) n_commit += nc;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (do_stats) s_ph[3] += __builtin_amdgcn_s_memtime() - r0t;
                    }
                    if (do_stats) s_round += __builtin_amdgcn_s_memtime() - t1;
                    i += nb;
                }
                if (reg_size < min_reg) continue;
                const unsigned long long tr0 = do_stats ? __builtin_amdgcn_s_memtime() : 0;
                if (do_stats) n_rpt += reg_size;
                // region2rect runs in lsd_rect_lanes_kernel (one lane per region): hand
                // over the region's points in queue order and its angle
                if (nout < kLsdRawCap) {
                    for (int j = lane; j < reg_size; j += 64) outP[npts + j] = q_get(g, j);
                    if (lane == 0) outR[nout] = LsdRegion{npts, reg_size, (double)reg_deg * kD2R};
                    npts += reg_size;
                    ++nout;
                } else {
                    overflow = true;
                }
                if (do_stats) s_rect += __builtin_amdgcn_s_memtime() - tr0;
            }
            if (pend) used_set_chunk(g, xb, y, pend, lane);
        }
    }
    if (lane == 0) {
        nlines[f * nOct + o] = nout;
        if (overflow) atomicOr(err + f, 4);
    }
    if (do_stats && lane == 0) {
        unsigned long long* S = stats + (size_t)(f * nOct + o) * 24;
        S[0] = __builtin_amdgcn_s_memtime() - t_begin;
        S[1] = s_setup; S[2] = s_round; S[3] = s_rect; S[4] = n_seed;
        S[5] = n_block; S[6] = n_round; S[7] = n_rpt; S[8] = n_commit;
        S[9] = s_ph[0]; S[10] = s_ph[1]; S[11] = s_ph[2]; S[12] = s_ph[3];
        S[13] = s_scan; S[14] = s_seed; S[15] = s_init;
        // where the wave ran: HW_ID (wave / SIMD / CU / SH / SE) and XCC_ID
        S[16] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        S[17] = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        S[18] = t_begin;
        S[19] = n_far; S[20] = n_spill;
        S[21] = t_real0;                                 // start and end on the chip-wide 100 MHz clock
        S[22] = __builtin_amdgcn_s_memrealtime();
    }
    if (!LOOP) break;  // one task per wave: the loop is a single trip
    }  // task
}

// ---------------------------------------------------------------------------
// LK3: region2rect (lsd.cpp:688-744) + get_theta (:746-782) with lane =
// region.  Each lane walks its own region's points in region order through
// the reference's three loops (centroid sums, inertia sums, l extents;
// lsd.cpp:697-744, :755-771): the identical sequence of double operations per
// region -- including the nine multiply-adds lsd.cpp.o fuses (x / y sums,
// Ixx / Iyy / Ixy, the eigenvalue root, l, the endpoints) -- with no LDS
// round trip and no idle lanes behind a serial lane 0.  Points and
// weights are fetched kRectU at a time so each lane keeps several loads in
// flight; regions of one wave are consecutive indices of one (frame, octave).
// ---------------------------------------------------------------------------
#ifndef PLVI_RECT_LANE_BLOCKS
#define PLVI_RECT_LANE_BLOCKS 2
#endif
constexpr int kRectLaneBlocks = PLVI_RECT_LANE_BLOCKS;  // 4-wave workgroups per (octave, frame), 256 regions each
// points fetched per group: 4 above kRectSmallNf frames (throughput, 64
// VGPRs); 16 for small batches, where the longest region's three serial
// passes are the launch (104 VGPRs; batch 64 7.97 -> 7.91 ms,
// profiles/r05/latency_ab.txt)
constexpr int kRectU = 4;
constexpr int kRectUSmall = 16;
constexpr int kRectSmallNf = 64;

template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(U <= 4 ? 8 : 1))) void lsd_rect_lanes_kernel(const LineOctDev* __restrict__ octs,
                                                             const double* __restrict__ modgrad,
                                                             const LsdRegion* __restrict__ regs,
                                                             const unsigned* __restrict__ regpts,
                                                             size_t regpts_frame, const int* __restrict__ nlines,
                                                             double prec, double scale_lsd,
                                                             LsdLine* __restrict__ lines, int oBase, int nOct) {
    // octaves oBase .. oBase + gridDim.z - 1 of nOct; grid (blocks, frames,
    // octaves): every frame's octave 0 (the most regions) is dispatched
    // before the octave-1 blocks, which fill the tail
    const int o = oBase + blockIdx.z, f = blockIdx.y;
    const int task = f * nOct + o;
    const int n = min(nlines[task], kLsdRawCap);
    const LineOctDev& od = octs[o];
    const int sw = od.sw;
    const double* M = modgrad + od.soff + (size_t)f * od.splane;
    const unsigned* P = regpts + (size_t)task * regpts_frame;
    for (int k = blockIdx.x * 256 + threadIdx.x; k - (int)(threadIdx.x & 63) < n; k += gridDim.x * 256) {
        if (k >= n) continue;
        const LsdRegion r = regs[(size_t)task * kLsdRawCap + k];
        const unsigned* q = P + r.start;
        const int rn = r.n;
        // centroid (lsd.cpp:697-705)
        double xs = 0.0, ys = 0.0, sum = 0.0;
        int i = 0;
        for (; i + U <= rn; i += U) {
            unsigned v[U];
            double w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = q[i + u];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = M[(size_t)(v[u] >> 16) * sw + (v[u] & 0xffffu)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                xs = rfma((double)(int)(v[u] & 0xffffu), w[u], xs);
                ys = rfma((double)(int)(v[u] >> 16), w[u], ys);
                sum += w[u];
            }
        }
        for (; i < rn; ++i) {
            const unsigned v = q[i];
            const double w = M[(size_t)(v >> 16) * sw + (v & 0xffffu)];
            xs = rfma((double)(int)(v & 0xffffu), w, xs);
            ys = rfma((double)(int)(v >> 16), w, ys);
            sum += w;
        }
        xs /= sum;
        ys /= sum;
        // inertia (get_theta, lsd.cpp:755-763)
        double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
        i = 0;
        for (; i + U <= rn; i += U) {
            unsigned v[U];
            double w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = q[i + u];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = M[(size_t)(v[u] >> 16) * sw + (v[u] & 0xffffu)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double dx = (double)(int)(v[u] & 0xffffu) - xs, dy = (double)(int)(v[u] >> 16) - ys;
                Ixx = rfma(dy * dy, w[u], Ixx);
                Iyy = rfma(dx * dx, w[u], Iyy);
                Ixy = rfma(-(dx * dy), w[u], Ixy);
            }
        }
        for (; i < rn; ++i) {
            const unsigned v = q[i];
            const double w = M[(size_t)(v >> 16) * sw + (v & 0xffffu)];
            const double dx = (double)(int)(v & 0xffffu) - xs, dy = (double)(int)(v >> 16) - ys;
            Ixx = rfma(dy * dy, w, Ixx);
            Iyy = rfma(dx * dx, w, Iyy);
            Ixy = rfma(-(dx * dy), w, Ixy);
        }
        const double lambda = 0.5 * (Ixx + Iyy - __builtin_sqrt(rfma(Ixx - Iyy, Ixx - Iyy, 4.0 * Ixy * Ixy)));
        double theta = (__builtin_fabs(Ixx) > __builtin_fabs(Iyy))
                           ? (double)plvi_fast_atan2((float)(lambda - Ixx), (float)Ixy)
                           : (double)plvi_fast_atan2((float)Ixy, (float)(lambda - Iyy));
        theta *= kD2R;
        if (angle_diff(theta, r.angle) > prec) theta += kPi;
        // dx = cos(theta), dy = sin(theta) (lsd.cpp:710-711): the reference
        // object calls glibc's sincos; its doubles feed l and the endpoints
        double dxv, dyv;
        plvi_sincos_glibc(theta, &dyv, &dxv);
        // l extents (lsd.cpp:722-735): order-free max(0, .) / min(0, .)
        double lmax = 0, lmin = 0;
        i = 0;
        for (; i + U <= rn; i += U) {
            unsigned v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = q[i + u];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double l = rfma((double)(int)(v[u] & 0xffffu) - xs, dxv, ((double)(int)(v[u] >> 16) - ys) * dyv);
                lmax = l > lmax ? l : lmax;
                lmin = l < lmin ? l : lmin;
            }
        }
        for (; i < rn; ++i) {
            const unsigned v = q[i];
            const double l = rfma((double)(int)(v & 0xffffu) - xs, dxv, ((double)(int)(v >> 16) - ys) * dyv);
            lmax = l > lmax ? l : lmax;
            lmin = l < lmin ? l : lmin;
        }
        double x1 = rfma(lmin, dxv, xs), y1 = rfma(lmin, dyv, ys);
        double x2 = rfma(lmax, dxv, xs), y2 = rfma(lmax, dyv, ys);
        x1 += 0.5; y1 += 0.5; x2 += 0.5; y2 += 0.5;
        if (scale_lsd != 1) {
            x1 /= scale_lsd; y1 /= scale_lsd; x2 /= scale_lsd; y2 /= scale_lsd;
        }
        lines[(size_t)task * kLsdRawCap + k] = LsdLine{(float)x1, (float)y1, (float)x2, (float)y2};
    }
}

// ---------------------------------------------------------------------------
// LK4: KeyLine assembly (LSDDetector_custom.cpp:306-346) + top-k filter
// (LineExtractor.cc:75-84: libstdc++ std::sort by response desc, truncate,
// class_id = i) + line equations (:106-115).  One workgroup per frame.
// ---------------------------------------------------------------------------
__device__ inline bool clip_line_ll(long long W, long long H, long long& x1, long long& y1, long long& x2,
                                    long long& y2) {
    int c1, c2;
    const long long right = W - 1, bottom = H - 1;
    if (W <= 0 || H <= 0) return false;
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        long long a;
        if (c1 & 12) {
            a = c1 < 8 ? 0 : bottom;
            x1 += (long long)((double)(a - y1) * (x2 - x1) / (y2 - y1));
            y1 = a;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            a = c2 < 8 ? 0 : bottom;
            x2 += (long long)((double)(a - y2) * (x2 - x1) / (y2 - y1));
            y2 = a;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                a = c1 == 1 ? 0 : right;
                y1 += (long long)((double)(a - x1) * (y2 - y1) / (x2 - x1));
                x1 = a;
                c1 = 0;
            }
            if (c2) {
                a = c2 == 1 ? 0 : right;
                y2 += (long long)((double)(a - x2) * (y2 - y1) / (x2 - x1));
                x2 = a;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

__device__ inline int line_iter_count(int W, int H, float fx1, float fy1, float fx2, float fy2) {
    int x1 = cv_round_f(fx1), y1 = cv_round_f(fy1), x2 = cv_round_f(fx2), y2 = cv_round_f(fy2);
    if ((unsigned)x1 >= (unsigned)W || (unsigned)x2 >= (unsigned)W || (unsigned)y1 >= (unsigned)H ||
        (unsigned)y2 >= (unsigned)H) {
        long long a = x1, b = y1, c = x2, d = y2;
        if (!clip_line_ll(W, H, a, b, c, d)) return 0;
        x1 = (int)a; y1 = (int)b; x2 = (int)c; y2 = (int)d;
    }
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    return max(dx, dy) + 1;
}

constexpr int kKlCap = 4096;  // keylines per frame before the top-k filter
static_assert(kKlCap <= kSortBlockMax, "std_sort_block packs 16-bit counts and positions");

__global__ __launch_bounds__(256) void line_assemble_kernel(const LineOctDev* __restrict__ octs, int nOct,
                                                            const LsdLine* __restrict__ lines,
                                                            const int* __restrict__ nlines, double min_length,
                                                            int nfeatures, int fcap, plvi_keyline* __restrict__ kl_out,
                                                            double* __restrict__ fn_out, int* __restrict__ count_out,
                                                            plvi_keyline* __restrict__ kl_tmp, int* __restrict__ err,
                                                            unsigned short* __restrict__ sort_pos) {
    __shared__ int s_scan[256];
    __shared__ int s_base;
    __shared__ __align__(8) SortItem s_items[kKlCap];
    const int f = blockIdx.x;
    plvi_keyline* tmp = kl_tmp + (size_t)f * kKlCap;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    for (int o = 0; o < nOct; ++o) {
        const LineOctDev& od = octs[o];
        const int n = nlines[f * nOct + o];
        const LsdLine* L = lines + (size_t)(f * nOct + o) * kLsdRawCap;
        const int W = od.w, H = od.h;
        for (int base = 0; base < n; base += 256) {
            const int k = base + threadIdx.x;
            plvi_keyline kl;
            int keep = 0;
            if (k < n) {
                float e0 = L[k].x1, e1 = L[k].y1, e2 = L[k].x2, e3 = L[k].y2;
                // checkLineExtremes (LSDDetector_custom.cpp:112-138)
                if (e0 < 0) e0 = 0;
                if (e0 >= W) e0 = (float)W - 1.0f;
                if (e2 < 0) e2 = 0;
                if (e2 >= W) e2 = (float)W - 1.0f;
                if (e1 < 0) e1 = 0;
                if (e1 >= H) e1 = (float)H - 1.0f;
                if (e3 < 0) e3 = 0;
                if (e3 >= H) e3 = (float)H - 1.0f;
                const double d0 = (double)(e0 - e2), d1 = (double)(e1 - e3);
                const double length = (float)__builtin_sqrt(d0 * d0 + d1 * d1);
                if (length > min_length) {
                    keep = 1;
                    const float os = od.octaveScale;
                    kl.startPointX = e0 * os;
                    kl.startPointY = e1 * os;
                    kl.endPointX = e2 * os;
                    kl.endPointY = e3 * os;
                    kl.sPointInOctaveX = e0;
                    kl.sPointInOctaveY = e1;
                    kl.ePointInOctaveX = e2;
                    kl.ePointInOctaveY = e3;
                    kl.lineLength = (float)length;
                    kl.numOfPixels = line_iter_count(W, H, e0, e1, e2, e3);
                    kl.angle = plvi_atan2f(kl.endPointY - kl.startPointY, kl.endPointX - kl.startPointX);
                    kl.octave = o;
                    kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
                    kl.response = kl.lineLength / (float)od.maxWH;
                    kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
                    kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
                }
            }
            s_scan[threadIdx.x] = keep;
            __syncthreads();
            for (int s = 1; s < 256; s <<= 1) {
                const int v = threadIdx.x >= s ? s_scan[threadIdx.x - s] : 0;
                __syncthreads();
                s_scan[threadIdx.x] += v;
                __syncthreads();
            }
            const int pos = s_base + s_scan[threadIdx.x] - keep;
            if (keep) {
                kl.class_id = pos;
                if (pos < kKlCap) tmp[pos] = kl;
            }
            __syncthreads();
            if (threadIdx.x == 0) s_base += s_scan[255];
            __syncthreads();
        }
    }
    const int n = s_base;
    if (n > kKlCap) {
        if (threadIdx.x == 0) { count_out[f] = 0; atomicOr(err + f, 8); }
        return;
    }
    int nfinal = n;
    const bool truncate = n > nfeatures && nfeatures != 0;
    if (truncate) {
        nfinal = nfeatures;
        // LineExtractor.cc:75-84 sorts by response, descending, with libstdc++
        // std::sort.  Without equal keys among the kept lines (and the one
        // after them) any sort gives its order: a block-wide bitonic sort of
        // (response desc, index) keys, then a tie check; only a frame with
        // such a tie replays the std::sort restatement on one thread.
        int P = 256;
        while (P < n) P <<= 1;
        unsigned long long* K = reinterpret_cast<unsigned long long*>(s_items);
        for (int i = threadIdx.x; i < P; i += 256)
            K[i] = i < n ? ((0xFFFFFFFFull - (unsigned long long)__float_as_uint(tmp[i].response)) << 32) |
                               (unsigned)i
                         : ~0ull;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = threadIdx.x; t < P / 2; t += 256) {
                    const int i = (t / j) * 2 * j + (t % j), ixj = i + j;
                    const bool asc = (i & k) == 0;
                    const unsigned long long x = K[i], y = K[ixj];
                    if ((x > y) == asc) {
                        K[i] = y;
                        K[ixj] = x;
                    }
                }
                __syncthreads();
            }
        bool tie = false;
        for (int i = threadIdx.x; i < nfinal && i + 1 < n; i += 256) tie |= (K[i] >> 32) == (K[i + 1] >> 32);
        if (__syncthreads_or(tie)) {
            __shared__ SortRange s_rng[2][256];
            __shared__ unsigned s_seg[kKlCap / 32];
            __shared__ int s_ctl[4];
            for (int i = threadIdx.x; i < n; i += 256) s_items[i] = SortItem{tmp[i].response, i};
            __syncthreads();
            // the libstdc++ std::sort permutation, replayed by the whole block
            // (std_sort.h: std_sort_block; long ranges partitioned by the
            // block, their stop positions in this frame's global scratch so the
            // LDS footprint -- and the kernel's occupancy -- stay as they were)
            unsigned short* sp = sort_pos + (size_t)f * 2 * kKlCap;
            std_sort_block(s_items, n, s_rng[0], s_rng[1], s_seg, s_ctl, sp, sp + kKlCap, s_scan);
        } else {
            for (int i = threadIdx.x; i < nfinal; i += 256) {
                const unsigned long long v = K[i];
                s_items[i] = SortItem{tmp[(int)(v & 0xffffffffu)].response, (int)(v & 0xffffffffu)};
            }
        }
        __syncthreads();
    }
    if (nfinal > fcap) {
        if (threadIdx.x == 0) { count_out[f] = 0; atomicOr(err + f, 8); }
        return;
    }
    plvi_keyline* outk = kl_out + (size_t)f * fcap;
    double* outf = fn_out + (size_t)f * fcap * 3;
    for (int i = threadIdx.x; i < nfinal; i += 256) {
        plvi_keyline kl = truncate ? tmp[s_items[i].idx] : tmp[i];
        if (truncate) kl.class_id = i;
        outk[i] = kl;
        // lineF = (sp x ep) / sqrt(l0^2 + l1^2), Eigen Vector3d (LineExtractor.cc:106-115)
        const double sx = kl.startPointX, sy = kl.startPointY, ex = kl.endPointX, ey = kl.endPointY;
        // LineExtractor.cc.o fuses sx*ey - sy*ex and a*a + b*b
        const double a = sy * 1.0 - 1.0 * ey, b = 1.0 * ex - sx * 1.0, c = rfma(sx, ey, -(sy * ex));
        const double nrm = __builtin_sqrt(rfma(a, a, b * b));
        outf[3 * i] = a / nrm;
        outf[3 * i + 1] = b / nrm;
        outf[3 * i + 2] = c / nrm;
    }
    if (threadIdx.x == 0) count_out[f] = nfinal;
}

// ---------------------------------------------------------------------------
// LB1: LBD octave 0 = GaussianBlur(5x5, 1) fixed point (taps t0,t1,t2,t1,t0 =
// 14,62,104 error-diffused, or 14,63,103 rounded: PLVI_COMPAT_GAUSS_ROUNDED)
// of the full frame (binary_descriptor_custom.cpp:359), Sobel dx/dy int16
// (:396-397).  LB2: octave 1 = pyrDown(blurred) (:367) + Sobel.  All
// borders reflect-101.
// ---------------------------------------------------------------------------
// LB1: one wave per column strip, lane
// L holds columns x0 - 4 + 4L .. +3 as one dword (lane 0 and the lane after
// the last output lane are halo), rows streamed top to bottom with 8 rows of
// loads in flight.  Vertical 5-tap first on the even / odd bytes in 16-bit
// fields (v_pk_mad_u16: fields never carry), horizontal 5-tap with
// v_dot2_u32_u16 on the lane's and its neighbours' field pairs (DPP), one
// rounding (exact integer sums, so the pass order is free).  Sobel from the
// last three blurred rows (reflect-101 of the blurred image at the borders:
// blurred row -1 = row 1, row h = row h - 2), again SWAR with the two
// neighbour columns from the adjacent lanes.
__device__ __forceinline__ uint32_t pk_madu16(uint32_t a, uint32_t b, uint32_t c) {  // per 16-bit field a*b+c
    typedef unsigned short u16v2 __attribute__((ext_vector_type(2)));
    const u16v2 r = __builtin_bit_cast(u16v2, a) * __builtin_bit_cast(u16v2, b) + __builtin_bit_cast(u16v2, c);
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t lb_dot2(uint32_t a, uint32_t b, uint32_t c) {  // a.lo*b.lo + a.hi*b.hi + c
    typedef unsigned short u16v2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16v2, a), __builtin_bit_cast(u16v2, b), c, false);
}
__device__ __forceinline__ uint32_t lb_ld4(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
constexpr int kLbOutLanes = 62;  // output lanes per strip (4 columns each)
#ifndef PLVI_LB_BANDS
#define PLVI_LB_BANDS 4
#endif
constexpr int kLbBands = PLVI_LB_BANDS;  // row bands per strip of lbd_sobel0_kernel (more waves per frame)

__global__ __launch_bounds__(64) void lbd_sobel0_kernel(const uint8_t* __restrict__ src, size_t s_frame, size_t s_row,
                                                        int w, int h, int strip_w, uint8_t* __restrict__ blur,
                                                        short2* __restrict__ go, size_t d_frame, int t0, int t1,
                                                        int t2) {
    const int f = blockIdx.y;
    const int lane = threadIdx.x;
    const int X0 = blockIdx.x * strip_w, X1 = min(X0 + strip_w, w);
    // row band [Y0, Y1) of gridDim.z bands: blurred rows from Y0 - 1 (the
    // Sobel of row Y0 needs it), input rows from Y0 - 3; reflection only at
    // the image's own top and bottom
    const int nb = gridDim.z, Y0 = (int)((long long)h * blockIdx.z / nb), Y1 = (int)((long long)h * (blockIdx.z + 1) / nb);
    if (Y1 <= Y0) return;
    const bool top = Y0 == 0, bottom = Y1 == h;
    const int c0 = X0 - 4 + 4 * lane;
    const bool need = c0 < X1 + 4;                      // output lanes and the two halo lanes
    const bool inner = need && c0 >= 0 && c0 + 4 <= w;  // a plain dword load
    const bool outl = lane >= 1 && c0 < X1;
    const int nout = min(4, X1 - c0);
    const uint8_t* S = src + (size_t)f * s_frame;
    uint8_t* Bp = blur + (size_t)f * d_frame;
    short2* Gp = go + (size_t)f * d_frame;
    auto load_row = [&](int r) -> uint32_t {
        const uint8_t* rp = S + (size_t)reflect101(r, h) * s_row;
        if (inner) return lb_ld4(rp + c0);
        uint32_t v = 0;
        if (need)
            for (int j = 0; j < 4; ++j) v |= (uint32_t)rp[reflect101(c0 + j, w)] << (8 * j);
        return v;
    };
    const uint32_t T0 = (uint32_t)t0 * 0x10001u, T1 = (uint32_t)t1 * 0x10001u, T2 = (uint32_t)t2 * 0x10001u;
    auto pk = [](int lo, int hi) { return (uint32_t)lo | (uint32_t)hi << 16; };
    // 5-row windows of even (c0, c0+2) / odd (c0+1, c0+3) bytes in 16-bit fields
    uint32_t pe[5] = {0, 0, 0, 0, 0}, po[5] = {0, 0, 0, 0, 0};
    uint32_t bm1 = 0, b0 = 0;  // blurred rows y-2, y-1 (4 bytes per lane)
    auto sobel_row = [&](int y, uint32_t bu, uint32_t bc, uint32_t bd) {
        // S(c) = up + 2 mid + down, D(c) = down - up, per 16-bit field (even / odd columns)
        const uint32_t ue = bu & 0x00ff00ffu, uo = (bu >> 8) & 0x00ff00ffu;
        const uint32_t me = bc & 0x00ff00ffu, mo = (bc >> 8) & 0x00ff00ffu;
        const uint32_t de = bd & 0x00ff00ffu, dd = (bd >> 8) & 0x00ff00ffu;
        const uint32_t Se = ue + 2 * me + de, So = uo + 2 * mo + dd;            // fields <= 1020
        const uint32_t De = de + 0x00ff00ffu - ue, Do = dd + 0x00ff00ffu - uo;  // D + 255, fields <= 510
        const uint32_t Sol = (uint32_t)dpp_from_left((int)So), Ser = (uint32_t)dpp_from_right((int)Se);
        const uint32_t Dol = (uint32_t)dpp_from_left((int)Do), Der = (uint32_t)dpp_from_right((int)De);
        const int gx0 = (int)(So & 0xffffu) - (int)(Sol >> 16), gx1 = (int)(Se >> 16) - (int)(Se & 0xffffu);
        const int gx2 = (int)(So >> 16) - (int)(So & 0xffffu), gx3 = (int)(Ser & 0xffffu) - (int)(Se >> 16);
        // gy(c) = D(c-1) + 2 D(c) + D(c+1) (offsets: 4 * 255)
        const int gy0 = (int)(Dol >> 16) + 2 * (int)(De & 0xffffu) + (int)(Do & 0xffffu) - 1020;
        const int gy1 = (int)(De & 0xffffu) + 2 * (int)(Do & 0xffffu) + (int)(De >> 16) - 1020;
        const int gy2 = (int)(Do & 0xffffu) + 2 * (int)(De >> 16) + (int)(Do >> 16) - 1020;
        const int gy3 = (int)(De >> 16) + 2 * (int)(Do >> 16) + (int)(Der & 0xffffu) - 1020;
        if (!outl || y < Y0 || y >= Y1) return;
        short2* o = Gp + (size_t)y * w + c0;
        const short2 g4[4] = {make_short2((short)gx0, (short)gy0), make_short2((short)gx1, (short)gy1),
                              make_short2((short)gx2, (short)gy2), make_short2((short)gx3, (short)gy3)};
        if (nout == 4 && (w & 3) == 0) {
            *reinterpret_cast<int4*>(o) = *reinterpret_cast<const int4*>(g4);
        } else {
            for (int j = 0; j < nout; ++j) o[j] = g4[j];
        }
    };
    const int rS = top ? -2 : Y0 - 3, rE = bottom ? h + 2 : Y1 + 3;
    const int yS = top ? 0 : Y0 - 1;
    uint32_t pv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] = rS + k < rE ? load_row(rS + k) : 0u;
    for (int rb = rS; rb < rE; rb += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = rb + k;
            if (r >= rE) break;
            const uint32_t V = pv[k];
            if (r + 8 < rE) pv[k] = load_row(r + 8);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                pe[q] = pe[q + 1];
                po[q] = po[q + 1];
            }
            pe[4] = V & 0x00ff00ffu;
            po[4] = (V >> 8) & 0x00ff00ffu;
            const int y = r - 2;  // blurred row from rows y-2 .. y+2
            if (y < yS) continue;
            // vertical: E = (c0, c0+2), O = (c0+1, c0+3); fields <= 255 * 256
            const uint32_t E = pk_madu16(T0, pe[0] + pe[4], pk_madu16(T1, pe[1] + pe[3], pk_madu16(T2, pe[2], 0u)));
            const uint32_t O = pk_madu16(T0, po[0] + po[4], pk_madu16(T1, po[1] + po[3], pk_madu16(T2, po[2], 0u)));
            const uint32_t El = (uint32_t)dpp_from_left((int)E), Ol = (uint32_t)dpp_from_left((int)O);
            const uint32_t Er = (uint32_t)dpp_from_right((int)E), Or = (uint32_t)dpp_from_right((int)O);
            // El = (c0-4, c0-2), Ol = (c0-3, c0-1), Er = (c0+4, c0+6), Or = (c0+5, c0+7)
            const uint32_t h0 = lb_dot2(El, pk(0, t0), lb_dot2(Ol, pk(0, t1), lb_dot2(E, pk(t2, t0), lb_dot2(O, pk(t1, 0), 0u))));
            const uint32_t h1 = lb_dot2(Ol, pk(0, t0), lb_dot2(E, pk(t1, t1), lb_dot2(O, pk(t2, t0), 0u)));
            const uint32_t h2 = lb_dot2(E, pk(t0, t2), lb_dot2(O, pk(t1, t1), lb_dot2(Er, pk(t0, 0), 0u)));
            const uint32_t h3 = lb_dot2(O, pk(t0, t2), lb_dot2(E, pk(0, t1), lb_dot2(Er, pk(t1, 0), lb_dot2(Or, pk(t0, 0), 0u))));
            const uint32_t Bv = min((h0 + 32768u) >> 16, 255u) | min((h1 + 32768u) >> 16, 255u) << 8 |
                                min((h2 + 32768u) >> 16, 255u) << 16 | min((h3 + 32768u) >> 16, 255u) << 24;
            if (outl && y >= Y0 && y < Y1) {
                uint8_t* o = Bp + (size_t)y * w + c0;
                if (nout == 4 && (w & 3) == 0) {
                    *reinterpret_cast<uint32_t*>(o) = Bv;
                } else {
                    for (int j = 0; j < nout; ++j) o[j] = (uint8_t)(Bv >> (8 * j));
                }
            }
            // Sobel row y - 1 (needs blurred rows y-2 .. y; row -1 = row 1)
            if (top && y == 1) sobel_row(0, Bv, b0, Bv);
            else if (y >= yS + 2) sobel_row(y - 1, bm1, b0, Bv);
            bm1 = b0;
            b0 = Bv;
        }
    }
    if (bottom) {
        if (h >= 2) sobel_row(h - 1, bm1, b0, bm1);  // row h = row h - 2
        else sobel_row(0, b0, b0, b0);
    }
}

// LB2: pyrDown(blurred octave 0) + Sobel.
// One wave per column strip of the output, lane L holds output columns
// xa = X0 - 2 + 2L, xa + 1 and the four source columns 2xa .. 2xa + 3 (one
// dword); source rows streamed, each pair of rows completes an output row.
// 1-4-6-4-1 vertical sums in 16-bit fields (<= 4080), horizontal with the
// left lane's two and the right lane's one column (DPP), (s + 128) >> 8.
// Sobel on the output with reflect-101 of the OUTPUT grid (P(-1) = P(1),
// P(w) = P(w - 2): the 2:1 grid is not symmetric about the far edge).
constexpr int kLb2OutLanes = 62;  // output lanes per strip (2 columns each)

__global__ __launch_bounds__(64) void lbd_sobel1_kernel(const uint8_t* __restrict__ blur0, int w0, int h0,
                                                        size_t s_frame, int w, int h, int strip_w,
                                                        short2* __restrict__ go, size_t d_frame) {
    const int f = blockIdx.y;
    const int lane = threadIdx.x;
    const int X0 = blockIdx.x * strip_w, X1 = min(X0 + strip_w, w);
    const int xa = X0 - 2 + 2 * lane;
    const int c0 = 2 * xa;  // first source column of this lane
    const bool need = xa < X1 + 2;
    const bool inner = need && c0 >= 0 && c0 + 4 <= w0;
    const bool out0 = lane >= 1 && xa < X1, out1 = lane >= 1 && xa + 1 < X1;
    const uint8_t* S = blur0 + (size_t)f * s_frame;
    short2* Gp = go + (size_t)f * d_frame;
    auto load_row = [&](int r) -> uint32_t {
        const uint8_t* rp = S + (size_t)reflect101(r, h0) * w0;
        if (inner) return lb_ld4(rp + c0);
        uint32_t v = 0;
        if (need)
            for (int j = 0; j < 4; ++j) v |= (uint32_t)rp[reflect101(c0 + j, w0)] << (8 * j);
        return v;
    };
    uint32_t pe[5] = {0, 0, 0, 0, 0}, po[5] = {0, 0, 0, 0, 0};
    int pm1 = 0, p0 = 0;  // output rows y-2, y-1: columns xa (bits 0-7) and xa+1 (bits 8-15)
    const bool xl = xa == 0, xr = xa + 1 == w - 1;  // output-grid reflection at the borders
    auto sobel_row = [&](int y, int up, int mid, int dn) {
        const int su = up & 255, su1 = up >> 8, sm = mid & 255, sm1 = mid >> 8, sd = dn & 255, sd1 = dn >> 8;
        const int S0 = su + 2 * sm + sd, S1 = su1 + 2 * sm1 + sd1;  // columns xa, xa + 1
        const int D0 = sd - su, D1 = sd1 - su1;
        const int pk = S1 | (D1 + 1024) << 12, pkl = S0 | (D0 + 1024) << 12;
        const int L = dpp_from_left(pk);    // column xa - 1 (left lane's xa + 1)
        const int R = dpp_from_right(pkl);  // column xa + 2 (right lane's xa)
        const int Sl = xl ? S1 : (L & 4095), Dl = xl ? D1 : (L >> 12) - 1024;
        const int Sr = xr ? S0 : (R & 4095), Dr = xr ? D0 : (R >> 12) - 1024;
        // column xa the last one (odd w): its right neighbour P(w) = P(w - 2)
        const bool last0 = xa + 1 >= w;
        const int Sr0 = last0 ? Sl : S1, Dr0 = last0 ? Dl : D1;
        const int gx0 = Sr0 - Sl, gy0 = Dl + 2 * D0 + Dr0;
        const int gx1 = Sr - S0, gy1 = D0 + 2 * D1 + Dr;
        short2* o = Gp + (size_t)y * w + xa;
        if (out0) o[0] = make_short2((short)gx0, (short)gy0);
        if (out1) o[1] = make_short2((short)gx1, (short)gy1);
    };
    uint32_t pv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] = load_row(k - 2);
    const int rend = 2 * h + 3;  // source rows -2 .. 2h
    for (int rb = -2; rb < rend - 2; rb += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = rb + k;
            if (r > 2 * h) break;
            const uint32_t V = pv[k];
            if (r + 8 <= 2 * h) pv[k] = load_row(r + 8);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                pe[q] = pe[q + 1];
                po[q] = po[q + 1];
            }
            pe[4] = V & 0x00ff00ffu;
            po[4] = (V >> 8) & 0x00ff00ffu;
            if ((k & 1) || r < 2) continue;  // output row y = (r - 2) / 2 from source rows 2y-2 .. 2y+2
            const int y = (r - 2) >> 1;
            // vertical 1-4-6-4-1: Ve = (c0, c0+2), Vo = (c0+1, c0+3), fields <= 4080
            const uint32_t Ve = pe[0] + pe[4] + 4 * (pe[1] + pe[3]) + 6 * pe[2];
            const uint32_t Vo = po[0] + po[4] + 4 * (po[1] + po[3]) + 6 * po[2];
            const uint32_t Vel = (uint32_t)dpp_from_left((int)Ve), Vol = (uint32_t)dpp_from_left((int)Vo);
            const uint32_t Ver = (uint32_t)dpp_from_right((int)Ve);
            // xa: columns c0-2 .. c0+2; xa+1: c0 .. c0+4
            const uint32_t s0 = (Vel >> 16) + 4 * (Vol >> 16) + 6 * (Ve & 0xffffu) + 4 * (Vo & 0xffffu) + (Ve >> 16);
            const uint32_t s1 = (Ve & 0xffffu) + 4 * (Vo & 0xffffu) + 6 * (Ve >> 16) + 4 * (Vo >> 16) + (Ver & 0xffffu);
            const int P = (int)((s0 + 128u) >> 8) | (int)((s1 + 128u) >> 8) << 8;
            if (y == 1) sobel_row(0, P, p0, P);
            else if (y >= 2) sobel_row(y - 1, pm1, p0, P);
            pm1 = p0;
            p0 = P;
        }
    }
    if (h >= 2) sobel_row(h - 1, pm1, p0, pm1);
    else sobel_row(0, p0, p0, p0);
}

// ---------------------------------------------------------------------------
// LB3: BinaryDescriptor::computeLBD (binary_descriptor_custom.cpp:1073-1342)
// + binaryConversion (:402-414, :663-667).  One wave per keyline: lane h
// walks support-region row h (63 rows) with the reference's sequential
// float stepping; lane 0 then accumulates the bands in row order and
// normalises.  Gaussian coefficient tables come from the host (double exp,
// cast to float at use, :1189/:1203).
// ---------------------------------------------------------------------------
__constant__ float c_gaussG[63];
__constant__ float c_gaussL[21];
__constant__ unsigned char c_comb[64];

__global__ __launch_bounds__(64) void lbd_describe_kernel(const LineOctDev* __restrict__ octs,
                                                          const short2* __restrict__ g_all,
                                                          const plvi_keyline* __restrict__ kls,
                                                          const int* __restrict__ counts, int fcap,
                                                          uint8_t* __restrict__ desc) {
    __shared__ float rq[8][64];
    __shared__ float bs[72];
    __shared__ float dv[72];
    const int li = blockIdx.x, f = blockIdx.y;
    if (li >= counts[f]) return;
    const plvi_keyline kl = kls[(size_t)f * fcap + li];
    const LineOctDev& od = octs[kl.octave];
    const short2* pg = g_all + od.loff + (size_t)f * od.lplane;  // (dx, dy) interleaved
    const short realWidth = (short)od.lw;
    const short imageWidth = realWidth - 1;
    const short imageHeight = (short)(od.lh - 1);
    const short lengthOfLSP = (short)kl.numOfPixels;
    const short halfWidth = (lengthOfLSP - 1) / 2;
    const short halfHeight = (63 - 1) / 2;
    const float mX = (float)(0.5 * (double)(kl.sPointInOctaveX + kl.ePointInOctaveX));
    const float mY = (float)(0.5 * (double)(kl.sPointInOctaveY + kl.ePointInOctaveY));
    const float dL0 = plvi_cosf(kl.angle), dL1 = plvi_sinf(kl.angle);
    const float dO0 = -dL1, dO1 = dL0;
    const int h = threadIdx.x;
    float pL = 0, nL = 0, pO = 0, nO = 0;
    // The coordinates are walked per row lane (reference order), but the
    // gathers are transposed through LDS: one gather instruction then covers
    // 8 rows x 8 consecutive samples instead of 64 rows at one sample, so its
    // lanes share cache lines (samples along a row are 1 px apart) and the
    // vector-memory path is not one cache line per lane
    // one array: each (row, sample) slot's index is read and its gathered
    // value written back by the same lane, and row lane h writes / reads only
    // its own row
    __shared__ int sidx[64][9];
    auto& sg = sidx;
    {
        float sX = -dL0 * halfWidth + dL1 * halfHeight + mX;
        float sY = -dL1 * halfWidth - dL0 * halfHeight + mY;
        for (int k = 0; k < h; ++k) {
            sX -= dL1;
            sY += dL0;
        }
        const int* pgi = reinterpret_cast<const int*>(pg);
        const int kk = h & 7, rr = h >> 3;
        for (int w0 = 0; w0 < lengthOfLSP; w0 += 8) {  // lengthOfLSP is wave-uniform
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                short t = (short)__builtin_roundf(sX);
                const short xc = (t < 0) ? 0 : (t > imageWidth) ? imageWidth : t;
                t = (short)__builtin_roundf(sY);
                const short yc = (t < 0) ? 0 : (t > imageHeight) ? imageHeight : t;
                sidx[h][k] = yc * realWidth + xc;
                sX += dL0;
                sY += dL1;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            int gv[8];
            const bool okk = w0 + kk < lengthOfLSP;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int r = 8 * i + rr;
                gv[i] = (r < 63 && okk) ? pgi[sidx[r][kk]] : 0;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) sg[8 * i + rr][kk] = gv[i];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (h < 63) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (w0 + k >= lengthOfLSP) break;
                    const short2 g = __builtin_bit_cast(short2, sg[h][k]);
                    const short dx = g.x, dy = g.y;
                    const float gDL = dx * dL0 + dy * dL1;
                    const float gDO = dx * dO0 + dy * dO1;
                    if (gDL > 0) pL += gDL;
                    else nL -= gDL;
                    if (gDO > 0) pO += gDO;
                    else nO -= gDO;
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
    }
    // row sums scaled by gaussCoefG_ (:1189-1197), per row lane
    if (h < 63) {
        const float c = c_gaussG[h];
        const float pLr = c * pL, nLr = c * nL, pOr = c * pO, nOr = c * nO;
        rq[0][h] = pLr; rq[1][h] = nLr; rq[2][h] = pLr * pLr; rq[3][h] = nLr * nLr;
        rq[4][h] = pOr; rq[5][h] = nOr; rq[6][h] = pOr * pOr; rq[7][h] = nOr * nOr;
    }
    __syncthreads();
    // band sums (:1202-1241): accumulator (band b, quantity q) takes the rows of
    // bands b-1, b, b+1 in row order, exactly the reference's += sequence for it
    for (int a = h; a < 72; a += 64) {
        const int b = a >> 3, q = a & 7;
        const bool sq = (q & 2) != 0;
        float acc = 0.f;
        const int r0 = max(0, 7 * (b - 1)), r1 = min(62, 7 * (b + 2) - 1);
        for (int r = r0; r <= r1; ++r) {
            const int j = r / 7, m = r - 7 * j;
            const float c = j == b ? c_gaussL[m + 7] : j == b + 1 ? c_gaussL[m + 14] : c_gaussL[m];
            const float x = rq[q][r];
            acc += sq ? c * c * x : c * x;
        }
        bs[a] = acc;
    }
    __syncthreads();
    if (h < 36) {  // mean / std per band (:1254-1281)
        const int b = h >> 2, k = h & 3;
        const int qs = (k < 2 ? 0 : 4) + (k & 1);
        const float invN = (b == 0 || b == 8) ? (float)(1.0 / (7 * 2.0)) : (float)(1.0 / (7 * 3.0));
        const float t = bs[8 * b + qs] * invN;
        dv[8 * b + k] = t;
        dv[8 * b + 4 + k] = __builtin_sqrtf(bs[8 * b + qs + 2] * invN - t * t);
    }
    __syncthreads();
    // normalisation (:1283-1330): the three sums stay sequential (lane 0),
    // the element-wise scaling and the 0.4 clip run on all lanes
    __shared__ float s_t[3];
    if (h == 0) {
        float tM = 0, tS = 0;
        for (int b = 0; b < 9; ++b) {
            const float* v = dv + 8 * b;
            tM += v[0] * v[0]; tM += v[1] * v[1]; tM += v[2] * v[2]; tM += v[3] * v[3];
            tS += v[4] * v[4]; tS += v[5] * v[5]; tS += v[6] * v[6]; tS += v[7] * v[7];
        }
        s_t[0] = 1 / __builtin_sqrtf(tM);
        s_t[1] = 1 / __builtin_sqrtf(tS);
    }
    __syncthreads();
    for (int i = h; i < 72; i += 64) {
        float v = dv[i] * ((i & 7) < 4 ? s_t[0] : s_t[1]);
        if ((double)v > 0.4) v = (float)0.4;
        dv[i] = v;
    }
    __syncthreads();
    if (h == 0) {
        float t = 0;
        for (int i = 0; i < 72; ++i) t += dv[i] * dv[i];
        s_t[2] = 1 / __builtin_sqrtf(t);
    }
    __syncthreads();
    for (int i = h; i < 72; i += 64) dv[i] = dv[i] * s_t[2];
    __syncthreads();
    if (h < 32) {
        const float* f1 = dv + 8 * c_comb[2 * h];
        const float* f2 = dv + 8 * c_comb[2 * h + 1];
        unsigned r = 0;
        for (int i = 0; i < 8; ++i)
            if (f1[i] > f2[i]) r += 1u << i;
        desc[((size_t)f * fcap + li) * 32 + h] = (uint8_t)r;
    }
}

}  // namespace plvi

