// oracle/cvprim.cpp — TEST INFRASTRUCTURE ONLY.  See cvprim.h.
// Restates the OpenCV 4.2 primitives named in SURVEY.md Appendix A.
// Compiled with -ffp-contract=off (the reference and OpenCV's baseline code
// contract no FMAs: SURVEY.md B.4).
#include "cvprim.h"

#include <algorithm>
#include <cassert>

namespace oracle {

// ---------------------------------------------------------------- A.5
// OpenCV 4.2 core/src/mathfuncs_core.simd.hpp atan_f32 (scalar path).
static const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------------------------- A.1/A.2
// cv::resize INTER_LINEAR, CV_8UC1 (imgproc/src/resize.cpp, OpenCV 4.2):
// scale exactly 2 → INTER_AREA fast path (ResizeAreaFastVec_SIMD_8u: the
// 128-bit SIMD body does (a+b+c+d+2)>>2 on the first floor(w/8)*8 columns,
// the scalar tail saturate_cast<uchar>(sum*0.25f)); otherwise the generic
// fixed-point bilinear path (HResizeLinear + VResizeLinear<uchar,int,short>).
static void resize_area2_u8(const ImageU8& src, ImageU8& dst) {
    const int dw = dst.w, dh = dst.h;
    const int dwidth1 = src.w / 2;
    const int simd = (dwidth1 / 8) * 8;
    for (int dy = 0; dy < dh; ++dy) {
        int sy0 = dy * 2;
        uint8_t* D = dst.row(dy);
        if (sy0 >= src.h) { std::fill(D, D + dw, 0); continue; }
        int w = (sy0 + 2 <= src.h) ? dwidth1 : 0;
        const uint8_t* S0 = src.row(sy0);
        const uint8_t* S1 = (sy0 + 1 < src.h) ? src.row(sy0 + 1) : S0;
        int dx = 0;
        for (; dx < std::min(simd, w); ++dx) {
            int s = S0[2 * dx] + S0[2 * dx + 1] + S1[2 * dx] + S1[2 * dx + 1];
            D[dx] = (uint8_t)std::min((s + 2) >> 2, 255);
        }
        for (; dx < w; ++dx) {
            int s = S0[2 * dx] + S0[2 * dx + 1] + S1[2 * dx] + S1[2 * dx + 1];
            D[dx] = (uint8_t)std::min(std::max(cv_round((float)s * 0.25f), 0), 255);
        }
        // Columns beyond src.w/2 only exist for odd widths, which never take
        // this path (is_area_fast requires an exact factor of 2).
        for (; dx < dw; ++dx) D[dx] = 0;
    }
}

void resize_linear_u8(const ImageU8& src, ImageU8& dst, int dw, int dh) {
    const int sw = src.w, sh = src.h;
    dst.create(dw, dh);
    if (dw == sw && dh == sh) { dst.px = src.px; return; }
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    const int iscale_x = cv_round(scale_x), iscale_y = cv_round(scale_y);
    const bool is_area_fast = std::fabs(scale_x - iscale_x) < DBL_EPSILON &&
                              std::fabs(scale_y - iscale_y) < DBL_EPSILON;
    if (is_area_fast && iscale_x == 2 && iscale_y == 2) { resize_area2_u8(src, dst); return; }

    const int ONE = 2048;  // INTER_RESIZE_COEF_SCALE
    std::vector<int> xofs(dw);
    std::vector<short> ialpha(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = (short)cv_round(c0 * ONE);
        ialpha[2 * dx + 1] = (short)cv_round(c1 * ONE);
    }
    std::vector<int> H0(dw), H1(dw);
    auto hresize = [&](const uint8_t* S, int* D) {
        int dx = 0;
        for (; dx < xmax; ++dx) {
            int sx = xofs[dx];
            D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
        }
        for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * ONE;
    };
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        short b0 = (short)cv_round((1.f - fy) * ONE), b1 = (short)cv_round(fy * ONE);
        int r0 = std::min(std::max(sy, 0), sh - 1);
        int r1 = std::min(std::max(sy + 1, 0), sh - 1);
        hresize(src.row(r0), H0.data());
        hresize(src.row(r1), H1.data());
        uint8_t* D = dst.row(dy);
        if (g_compat & 2) {
            // generic VResizeLinear + FixedPtCast<int, uchar, 22> (A.1 switch)
            for (int x = 0; x < dw; ++x)
                D[x] = (uint8_t)std::min(std::max((b0 * H0[x] + b1 * H1[x] + (1 << 21)) >> 22, 0), 255);
        } else {
            // VResizeLinear<uchar, int, short, FixedPtCast, VResizeLinearVec_32s8u>
            for (int x = 0; x < dw; ++x)
                D[x] = (uint8_t)((((b0 * (H0[x] >> 4)) >> 16) + ((b1 * (H1[x] >> 4)) >> 16) + 2) >> 2);
        }
    }
}

unsigned g_compat = 0;

// ---------------------------------------------------------------- A.6 exp
// OpenCV's exp64f (core/src/mathfuncs_core.simd.hpp; softfloat.cpp's f64_exp
// follows the same scheme): x * 64/ln2 rounded to an int v, 2^(v>>6) from
// the exponent bits, 2^((v&63)/64) * A0 from a 64-entry table, and a degree-5
// polynomial in the remainder.  Constants are the published decimal
// literals (confidence M: no OpenCV here to confirm them).
double cv_exp_table(double x) {
    const double A0s = .9670371139572337719125840413672004409288e-2;  // EXPPOLY_32F_A0
    struct Tab {
        double v[64];
        Tab(double a) { for (int i = 0; i < 64; ++i) v[i] = (double)exp2l((long double)i / 64.0L) * a; }
    };
    static const Tab tabs(A0s);  // thread-safe one-time init
    const double* tab = tabs.v;
    const double prescale = 1.4426950408889634073599246810019 * 64, postscale = 1. / 64;
    const double A5 = .99999999999999999998285227504999 / A0s, A4 = .69314718055994546743029643825322 / A0s,
                 A3 = .24022650695886477918181338054308 / A0s, A2 = .55504108793649567998466049042729e-1 / A0s,
                 A1 = .96180973140732918010002372686186e-2 / A0s, A0 = .13369713757180123244806654839424e-2 / A0s;
    double x0 = x * prescale;
    const int v = cv_round(x0);
    int t = (v >> 6) + 1023;
    t = !(t & ~2047) ? t : t < 0 ? 0 : 2047;
    uint64_t bits = (uint64_t)t << 52;
    double buf;
    std::memcpy(&buf, &bits, 8);
    x0 = (x0 - v) * postscale;
    return buf * tab[v & 63] * (((((A0 * x0 + A1) * x0 + A2) * x0 + A3) * x0 + A4) * x0 + A5);
}

// ---------------------------------------------------------------- A.4 / A.6
// getGaussianKernelBitExact (imgproc/src/smooth.dispatch.cpp) followed by
// getGaussianKernelFixedPoint_ED(.., 8).  exp: glibc (default; equals the
// correctly rounded exp at the configs' arguments) or OpenCV's table exp
// (g_compat & 4).  Parity vs real OpenCV unpinned.
static void gaussian_kernel_bitexact(int n, double sigma, std::vector<double>& res) {
    res.assign(n, 0.0);
    if (sigma <= 0) {
        static const double k3[] = {0.25, 0.5, 0.25};
        static const double k5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
        static const double k7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
        const double* k = n == 3 ? k3 : n == 5 ? k5 : n == 7 ? k7 : nullptr;
        if (n == 1) { res[0] = 1.0; return; }
        if (k) { for (int i = 0; i < n; ++i) res[i] = k[i]; return; }
        sigma = ((n - 1) * 0.5 - 1) * 0.3 + 0.8;  // mulAdd(n, 0.15, 0.35)
    }
    const double scale2X = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    std::vector<double> values(n2 + 1);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
        const double a = (double)(x * x) * scale2X;
        double t = (g_compat & 4) ? cv_exp_table(a) : std::exp(a);
        values[i] = t;
        sum += t;
    }
    sum *= 2;
    sum += 1.0;
    if ((n & 1) == 0) sum += 1.0;
    const double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; ++i) {
        double t = values[i] * mul1;
        res[i] = t;
        res[n - 1 - i] = t;
    }
    res[n2] = 1.0 * mul1;
    if ((n & 1) == 0) res[n2 + 1] = res[n2];
}

void gaussian_kernel_f64(int n, double sigma, double* k) {
    std::vector<double> r;
    gaussian_kernel_bitexact(n, sigma, r);
    for (int i = 0; i < n; ++i) k[i] = r[i];
}

void gaussian_taps_u8(int n, double sigma, int* taps) {
    std::vector<double> kd;
    gaussian_kernel_bitexact(n, sigma, kd);
    const int n2 = n / 2;
    if (g_compat & 1) {
        // plain rounding of every tap (the pre-error-diffusion conversion)
        for (int i = 0; i < n; ++i) taps[i] = (int)lrint(kd[i] * 256.0);
        return;
    }
    double err = 0;
    long sum = 0;
    for (int i = 0; i < n2; ++i) {
        double adj = kd[i] * 256.0 + err;
        long v0 = lrint(adj);
        err = adj - (double)v0;
        taps[i] = taps[n - 1 - i] = (int)v0;
        sum += v0;
    }
    taps[n2] = (int)(256 - 2 * sum);
}

void gaussian_blur_u8(const ImageU8& src, ImageU8& dst, int n, double sigma) {
    int k[16];
    gaussian_taps_u8(n, sigma, k);
    const int r = n / 2, w = src.w, h = src.h;
    std::vector<int> H((size_t)w * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t* S = src.row(y);
        for (int x = 0; x < w; ++x) {
            int s = 0;
            for (int i = 0; i < n; ++i) s += k[i] * S[reflect101(x + i - r, w)];
            H[(size_t)y * w + x] = s;
        }
    }
    ImageU8 out;
    out.create(w, h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            unsigned s = 0;
            for (int j = 0; j < n; ++j) s += (unsigned)(k[j] * H[(size_t)reflect101(y + j - r, h) * w + x]);
            out.row(y)[x] = (uint8_t)std::min((s + 32768u) >> 16, 255u);
        }
    dst = std::move(out);
}

// ---------------------------------------------------------------- A.3
// cv::FAST<16> cornerScore: d_k = v - p_k on the Bresenham circle of radius 3.
static const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                   {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

int fast_score(const uint8_t* p, int stride) {
    const int v = p[0];
    int d[16];
    for (int k = 0; k < 16; ++k) d[k] = v - p[kCircle[k][1] * stride + kCircle[k][0]];
    int best = -1000;
    for (int s = 0; s < 16; ++s) {
        int mn = 1000, mx = -1000;
        for (int i = 0; i < 9; ++i) {
            int t = d[(s + i) & 15];
            mn = std::min(mn, t);
            mx = std::max(mx, t);
        }
        best = std::max(best, std::max(mn, -mx));
    }
    return best;  // S; a corner at threshold t iff S > t, its score is S-1
}

// ---------------------------------------------------------------- A.7
void pyr_down_u8(const ImageU8& src, ImageU8& dst, int dw, int dh) {
    static const int k[5] = {1, 4, 6, 4, 1};
    ImageU8 out;
    out.create(dw, dh);
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x) {
            int s = 0;
            for (int j = 0; j < 5; ++j) {
                int sy = reflect101(2 * y + j - 2, src.h);
                int row = 0;
                for (int i = 0; i < 5; ++i) row += k[i] * src.at(reflect101(2 * x + i - 2, src.w), sy);
                s += k[j] * row;
            }
            out.row(y)[x] = (uint8_t)((s + 128) >> 8);
        }
    dst = std::move(out);
}

void sobel_s16(const ImageU8& src, std::vector<int16_t>& dx, std::vector<int16_t>& dy) {
    const int w = src.w, h = src.h;
    dx.assign((size_t)w * h, 0);
    dy.assign((size_t)w * h, 0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            int xm = reflect101(x - 1, w), xp = reflect101(x + 1, w);
            int ym = reflect101(y - 1, h), yp = reflect101(y + 1, h);
            int gx = (src.at(xp, ym) - src.at(xm, ym)) + 2 * (src.at(xp, y) - src.at(xm, y)) +
                     (src.at(xp, yp) - src.at(xm, yp));
            int gy = (src.at(xm, yp) - src.at(xm, ym)) + 2 * (src.at(x, yp) - src.at(x, ym)) +
                     (src.at(xp, yp) - src.at(xp, ym));
            dx[(size_t)y * w + x] = (int16_t)gx;
            dy[(size_t)y * w + x] = (int16_t)gy;
        }
}

}  // namespace oracle
