// tests/native/libm_device_check.hip — the product's glibc-faithful math
// (pl-vi-orbslam3_amd/csrc/plvi_math.h) as the gfx950 build evaluates it ON
// THE DEVICE (same compiler flags as the library: -O3 -ffp-contract=off)
// versus the HOST glibc the reference binary calls.
// tests/native/libm_check.cpp checks the same header compiled for the host;
// this checks the device code object (different compiler, builtins,
// denormal mode).
//
// usage: libm_device_check <mode> [n]
//   sincosf     every float bit pattern (2^32): plvi_sinf / plvi_cosf vs sinf / cosf
//   sincospos   every float in [0, 120): plvi_sincosf_pos vs sinf / cosf
//   lsdangles   every float deg in [0, 360]: float(plvi_cos/sin(+-deg*pi/180)) vs cos / sin
//   atan2f n    n seeded (y, x) pairs + grids: plvi_atan2f vs atan2f
//   fastatan2 n n seeded pairs + grid: plvi_fast_atan2 vs the oracle's cv::fastAtan2
//               (liboracle.so, oracle_fast_atan2)
//   r2rect      every float T in [0, 360]: plvi_sincos_glibc(θ) and (θ + pi),
//               θ = (double)T*pi/180, as doubles, bitwise vs glibc sincos
//               (region2rect, lsd.cpp:707-711)
// Prints "mismatches=<k> checked=<n>", exit 1 on any mismatch, 3 on a HIP error.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../pl-vi-orbslam3_amd/csrc/plvi_math.h"

extern "C" float oracle_fast_atan2(float y, float x);

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(3);                                                                \
        }                                                                           \
    } while (0)

// mode 0: sinf/cosf of bit pattern base+i; 1: sincosf_pos of bit pattern i;
// 2: float(cos/sin(+-deg*pi/180)) of bit pattern base+i (4 outputs);
// 3: atan2f(y[i], x[i]); 4: fast_atan2(y[i], x[i]);
// 5: sincos of θ and θ + pi as doubles (4 outputs, d0..d3)
__global__ void eval_kernel(int mode, uint32_t base, long n, const float* ya, const float* xa, float* o0, float* o1,
                            float* o2, float* o3, double* d0, double* d1, double* d2, double* d3) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 5) {
        double a = (double)plvi::u2f(base + (uint32_t)i) * (M_PI / 180);
        plvi::plvi_sincos_glibc(a, &d0[i], &d1[i]);
        a += M_PI;
        plvi::plvi_sincos_glibc(a, &d2[i], &d3[i]);
    } else if (mode == 0) {
        const float x = plvi::u2f(base + (uint32_t)i);
        o0[i] = plvi::plvi_sinf(x);
        o1[i] = plvi::plvi_cosf(x);
    } else if (mode == 1) {
        float s, c;
        plvi::plvi_sincosf_pos(plvi::u2f(base + (uint32_t)i), &s, &c);
        o0[i] = s;
        o1[i] = c;
    } else if (mode == 2) {
        const double a = (double)plvi::u2f(base + (uint32_t)i) * (M_PI / 180);
        o0[i] = (float)plvi::plvi_cos(a);
        o1[i] = (float)plvi::plvi_sin(a);
        o2[i] = (float)plvi::plvi_cos(-a);
        o3[i] = (float)plvi::plvi_sin(-a);
    } else if (mode == 3) {
        o0[i] = plvi::plvi_atan2f(ya[i], xa[i]);
    } else {
        o0[i] = plvi::plvi_fast_atan2(ya[i], xa[i]);
    }
}

static bool samed(double a, double b) { return plvi::d2u(a) == plvi::d2u(b); }

static bool same(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint32_t x, y;
    memcpy(&x, &a, 4);
    memcpy(&y, &b, 4);
    return x == y;
}

int main(int argc, char** argv) {
    const char* m = argc > 1 ? argv[1] : "sincosf";
    const int mode = !strcmp(m, "sincosf") ? 0 : !strcmp(m, "sincospos") ? 1 : !strcmp(m, "lsdangles") ? 2
                   : !strcmp(m, "atan2f") ? 3 : !strcmp(m, "fastatan2") ? 4 : !strcmp(m, "r2rect") ? 5 : -1;
    if (mode < 0) {
        fprintf(stderr, "unknown mode\n");
        return 2;
    }
    unsigned long long total;
    if (mode == 0) total = 1ull << 32;
    else if (mode == 1) total = plvi::f2u(120.0f);
    else if (mode == 2 || mode == 5) total = (unsigned long long)plvi::f2u(360.0f) + 1;
    else total = argc > 2 ? strtoull(argv[2], 0, 0) : 30000000ull;
    const long chunk = 1l << 26;
    const int nout = mode == 5 ? 0 : mode == 2 ? 4 : (mode <= 1 ? 2 : 1);
    const int ndout = mode == 5 ? 4 : 0;
    std::vector<float> h[4], ya, xa;
    std::vector<double> hd[4];
    float* d[4] = {nullptr, nullptr, nullptr, nullptr};
    double* dd[4] = {nullptr, nullptr, nullptr, nullptr};
    float *dy = nullptr, *dx = nullptr;
    for (int k = 0; k < nout; ++k) {
        h[k].resize(chunk);
        CK(hipMalloc(&d[k], chunk * sizeof(float)));
    }
    for (int k = 0; k < ndout; ++k) {
        hd[k].resize(chunk);
        CK(hipMalloc(&dd[k], chunk * sizeof(double)));
    }
    if (mode == 3 || mode == 4) {
        ya.resize(chunk);
        xa.resize(chunk);
        CK(hipMalloc(&dy, chunk * sizeof(float)));
        CK(hipMalloc(&dx, chunk * sizeof(float)));
    }
    int nt = std::thread::hardware_concurrency();
    if (nt > 16) nt = 16;  // the GPU box's CPU share per GPU
    std::atomic<unsigned long long> bad{0};
    unsigned long long checked = 0;
    std::mt19937_64 rng(mode == 3 ? 1234 : 99);
    std::uniform_int_distribution<uint32_t> bits;
    std::uniform_real_distribution<float> ur(mode == 3 ? -800.f : -4.f, mode == 3 ? 800.f : 4.f);
    for (unsigned long long off = 0; off < total; off += chunk) {
        const long n = (long)std::min<unsigned long long>(chunk, total - off);
        if (mode == 3 || mode == 4) {
            for (long i = 0; i < n; ++i) {
                const unsigned long long g = off + i;
                if (g % 3 == 0) { ya[i] = plvi::u2f(bits(rng)); xa[i] = plvi::u2f(bits(rng)); }
                else if (g % 3 == 1) { ya[i] = ur(rng); xa[i] = ur(rng); }
                else if (mode == 3) { ya[i] = (float)(int)ur(rng) * 0.5f; xa[i] = (float)(int)ur(rng) * 0.25f; }
                else { ya[i] = (float)((long)(g / 3) % 41 - 20); xa[i] = (float)((long)(g / 123) % 41 - 20); }
            }
            CK(hipMemcpy(dy, ya.data(), n * sizeof(float), hipMemcpyHostToDevice));
            CK(hipMemcpy(dx, xa.data(), n * sizeof(float), hipMemcpyHostToDevice));
        }
        hipLaunchKernelGGL(eval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, mode, (uint32_t)off, n, dy,
                           dx, d[0], d[1], d[2], d[3], dd[0], dd[1], dd[2], dd[3]);
        CK(hipGetLastError());
        for (int k = 0; k < nout; ++k) CK(hipMemcpy(h[k].data(), d[k], n * sizeof(float), hipMemcpyDeviceToHost));
        for (int k = 0; k < ndout; ++k) CK(hipMemcpy(hd[k].data(), dd[k], n * sizeof(double), hipMemcpyDeviceToHost));
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                unsigned long long b = 0;
                for (long i = t; i < n; i += nt) {
                    bool ok = true;
                    const float x = plvi::u2f((uint32_t)(off + i));
                    if (mode == 5) {
                        double a = (double)x * (M_PI / 180), gs, gc;
                        sincos(a, &gs, &gc);
                        ok = samed(hd[0][i], gs) && samed(hd[1][i], gc);
                        a += M_PI;
                        sincos(a, &gs, &gc);
                        ok = ok && samed(hd[2][i], gs) && samed(hd[3][i], gc);
                    } else if (mode == 0 || mode == 1) {
                        ok = same(h[0][i], sinf(x)) && same(h[1][i], cosf(x));
                    } else if (mode == 2) {
                        const double a = (double)x * (M_PI / 180);
                        ok = same(h[0][i], (float)std::cos(a)) && same(h[1][i], (float)std::sin(a)) &&
                             same(h[2][i], (float)std::cos(-a)) && same(h[3][i], (float)std::sin(-a));
                    } else if (mode == 3) {
                        ok = same(h[0][i], atan2f(ya[i], xa[i]));
                    } else {
                        ok = same(h[0][i], oracle_fast_atan2(ya[i], xa[i]));
                    }
                    if (!ok) {
                        if (b < 3) fprintf(stderr, "%s mismatch at %lld\n", m, (long long)(off + i));
                        ++b;
                    }
                }
                bad += b;
            });
        for (auto& x : th) x.join();
        checked += n;
    }
    printf("mismatches=%llu checked=%llu\n", (unsigned long long)bad, checked);
    return bad ? 1 : 0;
}
