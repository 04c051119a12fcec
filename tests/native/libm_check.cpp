// tests/native/libm_check.cpp — exhaustive / sampled comparison of the
// product's device math (pl-vi-orbslam3_amd/csrc/plvi_math.h, compiled here
// as host code with the same IEEE operations) against the HOST glibc, which
// is what the reference binary calls.  SURVEY.md B.3.
//
// usage: libm_check <mode> [lo_bits hi_bits]
//   sincosf     : every float bit pattern in [lo,hi) (default: all 2^32)
//   atan2f N    : N seeded random (y,x) pairs + edge grid
//   lsdangles   : every float deg in [0,360]: float(cos/sin((double)deg*pi/180))
//   sincospos   : branch-free sincosf vs glibc, every float in [0,120)
//   fastatan2 N : device cv::fastAtan2 vs the oracle's restatement, N pairs + grid
//   r2rect      : every float T in [0,360]: plvi_sincos_glibc(θ), θ = (double)T*pi/180
//                 and θ + pi, bitwise (double) vs glibc sincos
//   sincosd N   : plvi_sincos_glibc vs glibc sincos on N seeded doubles, |x| < 105414350
// Prints "mismatches=<k> checked=<n>" and exits non-zero on any mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>
#include <atomic>

#include "../../pl-vi-orbslam3_amd/csrc/plvi_math.h"
#include "../../oracle/cvprim.h"

static bool samed(double a, double b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    return plvi::d2u(a) == plvi::d2u(b);
}

static bool sincos_ok(double x) {
    double s, c, gs, gc;
    plvi::plvi_sincos_glibc(x, &s, &c);
    sincos(x, &gs, &gc);
    return samed(s, gs) && samed(c, gc);
}

static bool same(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint32_t x, y;
    memcpy(&x, &a, 4); memcpy(&y, &b, 4);
    return x == y;
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "sincosf";
    int nt = std::thread::hardware_concurrency();
    if (nt > 16) nt = 16;
    std::atomic<unsigned long long> bad{0}, checked{0};
    std::vector<std::thread> th;
    if (!strcmp(mode, "sincosf")) {
        unsigned long long lo = argc > 2 ? strtoull(argv[2], 0, 0) : 0ull;
        unsigned long long hi = argc > 3 ? strtoull(argv[3], 0, 0) : (1ull << 32);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                unsigned long long b = 0, c = 0;
                for (unsigned long long u = lo + t; u < hi; u += nt) {
                    float x = plvi::u2f((uint32_t)u);
                    if (!same(plvi::plvi_sinf(x), sinf(x))) { if (b < 5) fprintf(stderr, "sinf %a\n", x); ++b; }
                    if (!same(plvi::plvi_cosf(x), cosf(x))) { if (b < 5) fprintf(stderr, "cosf %a\n", x); ++b; }
                    ++c;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "atan2f")) {
        long n = argc > 2 ? atol(argv[2]) : 100000000L;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(1234 + t);
                std::uniform_real_distribution<float> u(-800.f, 800.f);
                std::uniform_int_distribution<uint32_t> bits;
                unsigned long long b = 0, c = 0;
                for (long i = t; i < n; i += nt) {
                    float y, x;
                    if (i % 3 == 0) { y = plvi::u2f(bits(rng)); x = plvi::u2f(bits(rng)); }
                    else if (i % 3 == 1) { y = u(rng); x = u(rng); }
                    else { y = (float)(int)u(rng) * 0.5f; x = (float)(int)u(rng) * 0.25f; }
                    if (!same(plvi::plvi_atan2f(y, x), atan2f(y, x))) {
                        if (b < 5) fprintf(stderr, "atan2f %a %a -> %a vs %a\n", y, x, plvi::plvi_atan2f(y, x), atan2f(y, x));
                        ++b;
                    }
                    ++c;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "lsdangles")) {
        const double D2R = M_PI / 180;
        uint32_t hi = plvi::f2u(360.0f);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                unsigned long long b = 0, c = 0;
                for (uint32_t u = t; u <= hi; u += nt) {
                    float deg = plvi::u2f(u);
                    double a = (double)deg * D2R;
                    // region_grow seed (lsd.cpp:648-649) and the float(angle)
                    // path of :678-679 (cosf/sinf of float(a)).
                    if (!same((float)plvi::plvi_cos(a), (float)std::cos(a))) { if (b < 5) fprintf(stderr, "cos %a\n", a); ++b; }
                    if (!same((float)plvi::plvi_sin(a), (float)std::sin(a))) { if (b < 5) fprintf(stderr, "sin %a\n", a); ++b; }
                    double na = -a;
                    if (!same((float)plvi::plvi_cos(na), (float)std::cos(na))) ++b;
                    if (!same((float)plvi::plvi_sin(na), (float)std::sin(na))) ++b;
                    ++c;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "sincospos")) {
        // branch-free sincosf of region_grow (lsd.cpp:678-679): every float in [0, 120)
        uint32_t hi = plvi::f2u(120.0f);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                unsigned long long b = 0, c = 0;
                for (uint32_t u = t; u < hi; u += nt) {
                    float x = plvi::u2f(u), s, co;
                    plvi::plvi_sincosf_pos(x, &s, &co);
                    if (!same(s, sinf(x)) || !same(co, cosf(x))) { if (b < 5) fprintf(stderr, "sincospos %a\n", x); ++b; }
                    ++c;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "r2rect")) {
        // region2rect (lsd.cpp:707-711): theta = fastAtan2(...) * DEG_TO_RADS,
        // + M_PI when it disagrees with the region angle, then sincos(theta)
        const double D2R = M_PI / 180;
        uint32_t hi = plvi::f2u(360.0f);
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                unsigned long long b = 0, c = 0;
                for (uint32_t u = t; u <= hi; u += nt) {
                    double a = (double)plvi::u2f(u) * D2R;
                    if (!sincos_ok(a)) { if (b < 5) fprintf(stderr, "r2rect %a\n", a); ++b; }
                    a += M_PI;
                    if (!sincos_ok(a)) { if (b < 5) fprintf(stderr, "r2rect+pi %a\n", a); ++b; }
                    c += 2;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "sincosd")) {
        long n = argc > 2 ? atol(argv[2]) : 100000000L;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(4321 + t);
                std::uniform_real_distribution<double> u1(-10.0, 10.0), u2(-105414349.0, 105414349.0);
                std::uniform_int_distribution<uint64_t> bits;
                unsigned long long b = 0, c = 0;
                for (long i = t; i < n; i += nt) {
                    double x;
                    if (i % 3 == 0) x = u1(rng);
                    else if (i % 3 == 1) x = u2(rng);
                    else {  // random bit patterns below 105414350 (all binades, denormals)
                        x = plvi::u2d(bits(rng));
                        if (!(std::fabs(x) < 105414349.0)) x = std::fmod(x, 105414349.0);
                        if (std::isnan(x)) x = 0.5;
                    }
                    if (!sincos_ok(x)) { if (b < 5) fprintf(stderr, "sincosd %a\n", x); ++b; }
                    ++c;
                }
                bad += b; checked += c;
            });
    } else if (!strcmp(mode, "fastatan2")) {
        long n = argc > 2 ? atol(argv[2]) : 100000000L;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 rng(99 + t);
                std::uniform_real_distribution<float> u(-4.f, 4.f);
                std::uniform_int_distribution<uint32_t> bits;
                unsigned long long b = 0, c = 0;
                for (long i = t; i < n; i += nt) {
                    float y, x;
                    if (i % 3 == 0) { y = plvi::u2f(bits(rng)); x = plvi::u2f(bits(rng)); }
                    else if (i % 3 == 1) { y = u(rng); x = u(rng); }
                    else { y = (float)((int)(i / 3) % 41 - 20); x = (float)((int)(i / 123) % 41 - 20); }
                    if (!same(plvi::plvi_fast_atan2(y, x), oracle::fast_atan2(y, x))) {
                        if (b < 5) fprintf(stderr, "fastatan2 %a %a\n", y, x);
                        ++b;
                    }
                    ++c;
                }
                bad += b; checked += c;
            });
    } else {
        fprintf(stderr, "unknown mode\n");
        return 2;
    }
    for (auto& x : th) x.join();
    printf("mismatches=%llu checked=%llu\n", (unsigned long long)bad, (unsigned long long)checked);
    return bad ? 1 : 0;
}
