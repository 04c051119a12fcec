// plvi_common.h — shared host/device helpers for the HIP front end.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../include/plvi_frontend.h"

#define PLVI_CHECK(expr)                                                                          \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "[plvi] HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, \
                    __LINE__, #expr);                                                             \
            return PLVI_E_HIP;                                                                    \
        }                                                                                         \
    } while (0)

namespace plvi {

constexpr int kWave = 64;

// LDS pointers carry address space 3 so every access is a ds_* instruction
// (a generic pointer turns them into flat accesses that wait on vmcnt too).
typedef unsigned __attribute__((address_space(3))) lds_u32;
typedef float __attribute__((address_space(3))) lds_f32;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef int __attribute__((address_space(3))) lds_i32;

__host__ __device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

// Global -> LDS staging of an h x w byte block by NT cooperating threads
// (thread t of NT), 8 loads in flight per thread: a plain element loop would
// wait for every load before its LDS store (one memory latency per element).
// Row/column from the flat index with an exact multiply-high division
// (m = ceil(2^32 / w) is exact for i < 2^32 / w).
template <int NT>
__device__ __forceinline__ void stage_bytes(uint8_t* __restrict__ dst, int dst_pitch, const uint8_t* __restrict__ src,
                                            size_t src_pitch, int w, int h, int t) {
    const int n = w * h;
    const unsigned m = (unsigned)(0xFFFFFFFFull / (unsigned)w) + 1u;
    for (int i0 = 0; i0 < n; i0 += 8 * NT) {
        uint8_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + t + k * NT;
            const int r = (int)__umulhi((unsigned)i, m), c = i - r * w;
            v[k] = i < n ? src[(size_t)r * src_pitch + c] : 0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + t + k * NT;
            const int r = (int)__umulhi((unsigned)i, m), c = i - r * w;
            if (i < n) dst[r * dst_pitch + c] = v[k];
        }
    }
}

// A device allocation owned by a pipeline (freed in the destructor).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int alloc(size_t n) {
        bytes = n;
        if (n == 0) return 0;
        return hipMalloc(&p, n) == hipSuccess ? 0 : PLVI_E_HIP;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

// Does a launch with `dyn` bytes of dynamic LDS fit the 160 KB of a CU? The
// kernel's static __shared__ data shares the budget (queried once per kernel).
template <auto Kernel>
inline bool lds_fits(size_t dyn) {
    static const size_t static_lds = [] {
        hipFuncAttributes fa{};
        return hipFuncGetAttributes(&fa, (const void*)Kernel) == hipSuccess ? fa.sharedSizeBytes : (size_t)1024;
    }();
    return dyn + static_lds <= 160 * 1024;
}

// Read and clear a pipeline's per-frame device error flags (orb_pipeline.hip).
int read_frame_errors(int* d_err, int nslots, int* frame_flags, int* any, hipStream_t st);

}  // namespace plvi
