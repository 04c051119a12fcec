// plvi_math.h — transcendental functions on the bit-exact path, restated so
// that device results equal the reference CPU's.
//
//   plvi_cosf / plvi_sinf : glibc 2.35 sysdeps/ieee754/flt-32 sinf/cosf
//       (sincosf.h), x86-64 FMA ifunc variant (every `a + b*c` of the C
//       source is one fused multiply-add; checked against the libm
//       disassembly).  Used by rBRIEF (src/ORBextractor.cc:111), LSD
//       region_grow (src/LSD/lsd.cpp:678-679) and LBD
//       (binary_descriptor_custom.cpp:1131-1132).
//   plvi_atan2f           : glibc flt-32 e_atan2f.c + s_atanf.c (fdlibm,
//       generic SSE2 build, no FMA).  KeyLine.angle
//       (LSDDetector_custom.cpp:336).
//   plvi_fast_atan2       : cv::fastAtan2 (OpenCV 4.2, degrees, no FMA).
//   plvi_cos / plvi_sin / plvi_sincos : double cos/sin for LSD region_grow's
//       seed (lsd.cpp:648-649), which only uses their float conversions:
//       fdlibm kernels with a 3-part Cody-Waite reduction (< 1 ulp), the
//       float conversions checked exhaustively against glibc over every
//       float angle LSD can produce (the doubles are not glibc's).
//   plvi_sincos_glibc     : glibc 2.35's double sincos itself (s_sincos.c,
//       SSE2 build), for region2rect (lsd.cpp:710-711), whose doubles feed
//       the endpoints: bitwise equal to glibc over region2rect's whole domain.
//
// Every function is __host__ __device__ so tests/native/libm_check.cpp can
// compare the very same code against the host glibc exhaustively.  All
// callers must be compiled with -ffp-contract=off.
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define PLVI_HD __host__ __device__ __forceinline__
#else
#define PLVI_HD static inline
#endif

namespace plvi {

PLVI_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
PLVI_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
PLVI_HD uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
PLVI_HD double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
PLVI_HD double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

// The reference's own sources are built by GCC 9.4 with `-O3 -march=native`
// (CMakeLists.txt; build/CMakeFiles/ORB_SLAM3-Relocalization.dir/flags.make)
// and GCC's C++ front end contracts `a*b + c` into one fused multiply-add
// even under -std=c++11.  The shipped objects show exactly which expressions
// were fused (tests/test_ref_objects.py pins every site on the path); those
// sites call rfma / rfmaf, everything else stays one IEEE op per operator
// (-ffp-contract=off).  For `a*b + c*d` GCC fuses the left product:
// rfma(a, b, c*d).
PLVI_HD double rfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
PLVI_HD float rfmaf(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// ------------------------------------------------------------ sinf / cosf
// __sincosf_table (values dumped from the glibc 2.35 libm used by the
// reference host).  Entry 1 = entry 0 with the cosine polynomial negated.
struct SinCosF {
    double c0, c1, s1, c2, s2, c3, s3, c4;
};
#define PLVI_HPI_INV 0x1.45f306dc9c883p+23
#define PLVI_HPI 0x1.921fb54442d18p+0
#define PLVI_PI63 0x1.921fb54442d18p-62

PLVI_HD SinCosF sincosf_tab(int k) {
    SinCosF t;
    t.c0 = 0x1.0p+0; t.c1 = -0x1.ffffffd0c621cp-2; t.s1 = -0x1.555545995a603p-3;
    t.c2 = 0x1.55553e1068f19p-5; t.s2 = 0x1.1107605230bc4p-7; t.c3 = -0x1.6c087e89a359dp-10;
    t.s3 = -0x1.994eb3774cf24p-13; t.c4 = 0x1.99343027bf8c3p-16;
    if (k) { t.c0 = -t.c0; t.c1 = -t.c1; t.c2 = -t.c2; t.c3 = -t.c3; t.c4 = -t.c4; }
    return t;
}

PLVI_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// sinf_poly (sincosf.h), FMA contraction as in __sinf_fma.
PLVI_HD float sinf_poly(double x, double x2, const SinCosF& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fmad(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = fmad(x3, p.s1, x);
        return (float)fmad(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = fmad(x2, p.c4, p.c3);
        double c1 = fmad(x2, p.c1, p.c0);
        double x6 = x4 * x2;
        double c = fmad(x4, p.c2, c1);
        return (float)fmad(x6, c2, c);
    }
}

// reduce_fast: !TOINT_INTRINSICS form, x - n*hpi fused (vfnmadd).
PLVI_HD double reduce_fast(double x, int* np) {
    double r = x * PLVI_HPI_INV;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fmad(-(double)n, PLVI_HPI, x);
}

PLVI_HD double reduce_large(uint32_t xi, int* np) {
    const uint32_t inv_pio4[24] = {0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44,
                                   0x6e4e4415, 0x4e441529, 0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1,
                                   0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db, 0xddc0db62,
                                   0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0x7fffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * PLVI_PI63;
}

PLVI_HD float plvi_sinf(float y) {
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sinf_poly(x, s, sincosf_tab(0), 0);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        double s = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, sincosf_tab((n & 2) ? 1 : 0), n);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        int q = (n + sign) & 3;
        double s = (q == 1 || q == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, sincosf_tab(((n + sign) & 2) ? 1 : 0), n);
    }
    return (y - y) / (y - y);
}

PLVI_HD float plvi_cosf(float y) {
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sinf_poly(x, x2, sincosf_tab(0), 1);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        double s = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, sincosf_tab((n & 2) ? 1 : 0), n ^ 1);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        int q = (n + sign) & 3;
        double s = (q == 1 || q == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, sincosf_tab(((n + sign) & 2) ? 1 : 0), n ^ 1);
    }
    return (y - y) / (y - y);
}

// sinf(y) and cosf(y) for 0 <= y < 120 without lane divergence (LSD feeds
// float(deg * DEG_TO_RADS), deg in [0, 360)).  For y < pi/4 glibc's direct
// branch equals the reduce_fast branch with n = 0 (x - 0*hpi == x exactly),
// so one reduction serves both; the sine and cosine polynomials are both
// evaluated once and selected by the quadrant parity.  Checked exhaustively
// against plvi_sinf/plvi_cosf and glibc (tests/native/libm_check.cpp).
PLVI_HD void plvi_sincosf_pos(float y, float* sp, float* cp) {
    int n;
    const double x = reduce_fast((double)y, &n);
    const double sg = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;
    const double neg = (n & 2) ? -1.0 : 1.0;
    const double xs = x * sg, x2 = x * x;
    // sine polynomial (s coefficients are not negated in table entry 1)
    const double x3 = xs * x2;
    const double s1 = fmad(x2, -0x1.994eb3774cf24p-13, 0x1.1107605230bc4p-7);
    const double x7 = x3 * x2;
    const double sv = fmad(x3, -0x1.555545995a603p-3, xs);
    const float S = (float)fmad(x7, s1, sv);
    // cosine polynomial (c coefficients negated in table entry 1)
    const double x4 = x2 * x2;
    const double c2 = fmad(x2, neg * 0x1.99343027bf8c3p-16, neg * -0x1.6c087e89a359dp-10);
    const double c1 = fmad(x2, neg * -0x1.ffffffd0c621cp-2, neg * 0x1.0p+0);
    const double x6 = x4 * x2;
    const double cv = fmad(x4, neg * 0x1.55553e1068f19p-5, c1);
    const float C = (float)fmad(x6, c2, cv);
    float s = (n & 1) ? C : S, c = (n & 1) ? S : C;
    if (abstop12(y) < abstop12(0x1p-12f)) { s = y; c = 1.0f; }
    *sp = s;
    *cp = c;
}

// ------------------------------------------------------------ fastAtan2
PLVI_HD float plvi_fast_atan2(float y, float x) {
    const float k = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;
    float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
    // both branches of cv::fastAtan2 share one division and one polynomial
    // (select form: no lane divergence, identical operations per branch)
    const bool ge = ax >= ay;
    const float c = (ge ? ay : ax) / ((ge ? ax : ay) + eps);
    const float c2 = c * c;
    const float pc = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    float a = ge ? pc : 90.f - pc;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ------------------------------------------------------------ atan2f
PLVI_HD float plvi_atanf_core(float x) {  // fdlibm s_atanf.c
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f,  -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f,  -3.6531571299e-02f, 1.6285819933e-02f};
    float w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)f2u(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        if (hx > 0) return atanhi[3] + atanlo[3];
        return -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = ((float)2.0 * x - 1.0f) / ((float)2.0 + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - (float)1.5) / (1.0f + (float)1.5 * x); }
            else { id = 3; x = -(float)1.0 / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}

PLVI_HD float plvi_atan2f(float y, float x) {  // fdlibm e_atan2f.c
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f;
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    float z;
    int32_t k, m, hx, hy, ix, iy;
    hx = (int32_t)f2u(x);
    ix = hx & 0x7fffffff;
    hy = (int32_t)f2u(y);
    iy = hy & 0x7fffffff;
    if ((ix > 0x7f800000) || (iy > 0x7f800000)) return x + y;
    if (hx == 0x3f800000) return plvi_atanf_core(y);
    m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return (float)3.0 * pi_o_4 + tiny;
                default: return (float)-3.0 * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
                case 0: return 0.0f;
                case 1: return -0.0f;
                case 2: return pi + tiny;
                default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + (float)0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else {
        z = plvi_atanf_core(__builtin_fabsf(y / x));
    }
    switch (m) {
        case 0: return z;
        case 1: return u2f(f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ------------------------------------------------------------ double sin/cos
PLVI_HD double k_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

PLVI_HD double k_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    uint32_t ix = (uint32_t)(d2u(x) >> 32) & 0x7fffffff;
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));
    double qx = ix > 0x3fe90000 ? 0.28125 : u2d((uint64_t)(ix - 0x00200000) << 32);
    double hz = 0.5 * z - qx;
    double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

// fdlibm __ieee754_rem_pio2 medium path (|x| < 2^20 * pi/2), 3 iterations.
PLVI_HD int rem_pio2(double x, double* y0, double* y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    double ax = __builtin_fabs(x);
    if (ax <= 0.78539816339744827900) { *y0 = x; *y1 = 0; return 0; }
    double fn = __builtin_rint(ax * invpio2);
    int n = (int)fn;
    double r = ax - fn * pio2_1;
    double w = fn * pio2_1t;
    uint32_t j = (uint32_t)(d2u(ax) >> 52) & 0x7ff;
    double y = r - w;
    int i = (int)j - (int)((d2u(y) >> 52) & 0x7ff);
    if (i > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y = r - w;
        i = (int)j - (int)((d2u(y) >> 52) & 0x7ff);
        if (i > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y = r - w;
        }
    }
    double yl = (r - y) - w;
    if (x < 0) { *y0 = -y; *y1 = -yl; return -n; }
    *y0 = y; *y1 = yl;
    return n;
}

PLVI_HD double plvi_sin(double x) {
    double y0, y1;
    int n = rem_pio2(x, &y0, &y1) & 3;
    switch (n) {
        case 0: return k_sin(y0, y1, 1);
        case 1: return k_cos(y0, y1);
        case 2: return -k_sin(y0, y1, 1);
        default: return -k_cos(y0, y1);
    }
}

PLVI_HD double plvi_cos(double x) {
    double y0, y1;
    int n = rem_pio2(x, &y0, &y1) & 3;
    switch (n) {
        case 0: return k_cos(y0, y1);
        case 1: return -k_sin(y0, y1, 1);
        case 2: return -k_cos(y0, y1);
        default: return k_sin(y0, y1, 1);
    }
}

// sin and cos of one argument together: one argument reduction, both kernels,
// quadrant by selects (no divergence across lanes with different quadrants).
// Bitwise equal to plvi_sin / plvi_cos.
PLVI_HD void plvi_sincos(double x, double* s, double* c) {
    double y0, y1;
    const int n = rem_pio2(x, &y0, &y1) & 3;
    const double ks = k_sin(y0, y1, 1), kc = k_cos(y0, y1);
    *s = n == 0 ? ks : n == 1 ? kc : n == 2 ? -ks : -kc;
    *c = n == 0 ? kc : n == 1 ? -ks : n == 2 ? -kc : ks;
}

// ------------------------------------------------------------ glibc sincos
// glibc 2.35 sysdeps/ieee754/dbl-64/s_sincos.c with s_sin.c's do_sin, do_cos,
// reduce_sincos and do_sincos (constants from usncs.h).  On x86-64 `sincos`
// is NOT an ifunc (unlike sin / cos, whose __sin_fma / __cos_fma contract
// multiply-adds): libm.so.6 exports one SSE2 build of it, no fused operation
// in its disassembly, so every operation below is one IEEE operation
// (callers build with -ffp-contract=off).  This is the call region2rect
// makes (src/LSD/lsd.cpp:710-711; the reference object calls sincos,
// tests/test_ref_objects.py), whose unrounded double results feed the l
// extents and the endpoints (:719, :729-732).  Bitwise equal to glibc's
// sincos over region2rect's domain (every θ = (double)T·π/180 for float T in
// [0, 360], and θ + π) on the host and on the device
// (tests/native/libm_check.cpp / libm_device_check.hip, mode r2rect) and on
// sampled doubles (mode sincosd).  Domain: |x| < 105414350 (glibc's
// __branred range is not restated).
constexpr double kGlibcSinCosTab[440] = {
#include "glibc_sincostab.inc"
};

PLVI_HD void glibc_tab(double u, double* sn, double* ssn, double* cs, double* ccs) {
    const int k = (int)(uint32_t)d2u(u) << 2;  // SINCOS_TABLE_LOOKUP: u.i[LOW_HALF] << 2
    *sn = kGlibcSinCosTab[k];
    *ssn = kGlibcSinCosTab[k + 1];
    *cs = kGlibcSinCosTab[k + 2];
    *ccs = kGlibcSinCosTab[k + 3];
}

#define PLVI_G_SN3 -0x1.5555555555515p-3
#define PLVI_G_SN5 0x1.11110e829872fp-7
#define PLVI_G_CS2 0x1.0p-1
#define PLVI_G_CS4 -0x1.5555555555535p-5
#define PLVI_G_CS6 0x1.6c16bedd9e239p-10
#define PLVI_G_BIG 0x1.8p+45

// do_cos (s_sin.c)
PLVI_HD double glibc_do_cos(double x, double dx) {
    if (x < 0) dx = -dx;
    const double u = PLVI_G_BIG + __builtin_fabs(x);
    x = __builtin_fabs(x) - (u - PLVI_G_BIG) + dx;
    const double xx = x * x;
    const double s = x + x * xx * (PLVI_G_SN3 + xx * PLVI_G_SN5);
    const double c = xx * (PLVI_G_CS2 + xx * (PLVI_G_CS4 + xx * PLVI_G_CS6));
    double sn, ssn, cs, ccs;
    glibc_tab(u, &sn, &ssn, &cs, &ccs);
    const double cor = (ccs - s * ssn - cs * c) - sn * s;
    return cs + cor;
}

// do_sin (s_sin.c), TAYLOR_SIN below 0.126
PLVI_HD double glibc_do_sin(double x, double dx) {
    const double xold = x;
    if (__builtin_fabs(x) < 0.126) {
        const double xx = x * x;
        // POLYNOMIAL(xx) = ((((s5*xx + s4)*xx + s3)*xx + s2)*xx) + s1
        const double p = ((((-0x1.addffc2fcdf59p-26 * xx + 0x1.71de27b9a7ed9p-19) * xx + -0x1.a01a019db08b8p-13) * xx +
                           0x1.1111111110ecep-7) * xx) + -0x1.5555555555555p-3;
        const double t = ((p * x - 0.5 * dx) * xx + dx);
        return x + t;
    }
    if (x <= 0) dx = -dx;
    const double u = PLVI_G_BIG + __builtin_fabs(x);
    x = __builtin_fabs(x) - (u - PLVI_G_BIG);
    const double xx = x * x;
    const double s = x + (dx + x * xx * (PLVI_G_SN3 + xx * PLVI_G_SN5));
    const double c = x * dx + xx * (PLVI_G_CS2 + xx * (PLVI_G_CS4 + xx * PLVI_G_CS6));
    double sn, ssn, cs, ccs;
    glibc_tab(u, &sn, &ssn, &cs, &ccs);
    const double cor = (ssn + s * ccs - sn * c) + cs * s;
    return __builtin_copysign(sn + cor, xold);
}

// reduce_sincos (s_sin.c): quadrant and a + da = x - n*pi/2
PLVI_HD int glibc_reduce(double x, double* a, double* da) {
    const double hpinv = 0x1.45f306dc9c883p-1, toint = 0x1.8p+52;
    const double mp1 = 0x1.921fb58000000p+0, mp2 = -0x1.dde973c000000p-27;
    const double pp3 = -0x1.cb3b398000000p-55, pp4 = -0x1.d747f23e32ed7p-83;
    const double t = (x * hpinv + toint);
    const double xn = t - toint;
    const int n = (int)((uint32_t)d2u(t) & 3);
    const double y = (x - xn * mp1) - xn * mp2;
    double t1 = xn * pp3;
    const double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * pp4;
    const double b = t2 - t1;
    db += (t2 - b) - t1;
    *a = b;
    *da = db;
    return n;
}

PLVI_HD double glibc_do_sincos(double a, double da, int n) {
    const double r = (n & 1) ? glibc_do_cos(a, da) : glibc_do_sin(a, da);
    return (n & 2) ? -r : r;
}

PLVI_HD void plvi_sincos_glibc(double x, double* sinx, double* cosx) {
    const uint32_t k = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
    if (k < 0x400368fdu) {
        if (k < 0x3e400000u) {
            *sinx = x;
            *cosx = 1.0;
            return;
        }
        if (k < 0x3feb6000u) {
            *sinx = glibc_do_sin(x, 0);
            *cosx = glibc_do_cos(x, 0);
            return;
        }
        const double hp0 = 0x1.921fb54442d18p+0, hp1 = 0x1.1a62633145c07p-54;
        const double y = hp0 - __builtin_fabs(x);
        const double a = y + hp1;
        const double da = (y - a) + hp1;
        *sinx = __builtin_copysign(glibc_do_cos(y, hp1), x);
        *cosx = glibc_do_sin(a, da);
        return;
    }
    double a, da;
    const int n = glibc_reduce(x, &a, &da);
    *sinx = glibc_do_sincos(a, da, n);
    *cosx = glibc_do_sincos(a, da, n + 1);
}

// cvRound (round half to even) and roundf (half away from zero).
PLVI_HD int cv_round_f(float v) { return (int)__builtin_rintf(v); }
PLVI_HD int cv_round_d(double v) { return (int)__builtin_rint(v); }

}  // namespace plvi
