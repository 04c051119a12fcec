// oracle/cvprim.h — TEST INFRASTRUCTURE ONLY (the checker, never the product).
//
// CPU restatement of the OpenCV 4.2 / glibc primitives that the reference's
// hot path calls.  OpenCV is not present in this image
// and no reference test pins these primitives, so every function here carries
// "parity unpinned" against real OpenCV: each follows the published OpenCV 4.2
// algorithm as restated in SURVEY.md Appendix A, locked by the KATs in
// tests/test_oracle_kat.py.  libm calls (cosf/sinf/atan2f/cos/sin/exp) go to
// the HOST glibc, exactly as the reference binary does.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this code.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle {

// Switches for the Appendix-A items no reference test pins (same bits as
// PLVI_COMPAT_* in include/plvi_frontend.h), process-global in the oracle:
//  1 = A.4 plainly rounded 8-bit Gaussian taps instead of error diffusion
//  2 = A.1 generic vertical fixed-point cast in resize INTER_LINEAR 8U
//  4 = A.6 OpenCV table + polynomial exp (exp64f) in getGaussianKernel
extern unsigned g_compat;
double cv_exp_table(double x);

// A.10 cvRound: round half to even (SSE cvtss2si / cvtsd2si).
static inline int cv_round(float v) { return (int)lrintf(v); }
static inline int cv_round(double v) { return (int)lrint(v); }
static inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }

// A.5 cv::fastAtan2 (OpenCV 4.2 mathfuncs_core, scalar, no FMA).  Degrees.
float fast_atan2(float y, float x);

// reflect-101 border index (BORDER_REFLECT_101 / BORDER_DEFAULT).
static inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    }
    return p;
}

struct ImageU8 {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
    uint8_t* row(int y) { return px.data() + (size_t)y * w; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
    void create(int W, int H) { w = W; h = H; px.assign((size_t)W * H, 0); }
};

// A.1 / A.2 cv::resize(src, dst, Size(dw,dh), 0, 0, INTER_LINEAR) for CV_8UC1.
void resize_linear_u8(const ImageU8& src, ImageU8& dst, int dw, int dh);

// A.4 cv::GaussianBlur(src, dst, Size(k,k), sigma) on a non-submatrix CV_8UC1:
// fixed-point separable filter with 8-fractional-bit taps (error diffusion).
void gaussian_taps_u8(int ksize, double sigma, int* taps);
void gaussian_blur_u8(const ImageU8& src, ImageU8& dst, int ksize, double sigma);

// A.6 getGaussianKernel(n, sigma, CV_64F) (bit-exact soft-double sequence).
void gaussian_kernel_f64(int n, double sigma, double* k);

// A.3 FAST-9/16 cornerScore closed form (score = S-1, independent of t for corners).
int fast_score(const uint8_t* p, int stride);  // returns S (= max arc contrast)

// A.7 pyrDown to (dw,dh) and Sobel 3x3 to int16, reflect-101.
void pyr_down_u8(const ImageU8& src, ImageU8& dst, int dw, int dh);
void sobel_s16(const ImageU8& src, std::vector<int16_t>& dx, std::vector<int16_t>& dy);

}  // namespace oracle
