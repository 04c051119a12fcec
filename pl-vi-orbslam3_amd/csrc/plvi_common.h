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

__host__ __device__ inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
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

}  // namespace plvi
