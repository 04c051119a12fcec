// capi.hip — library-level entry points of the C-ABI (include/plvi_frontend.h).
#include <hip/hip_runtime.h>

#include "plvi_common.h"

extern "C" const char* plvi_version(void) { return "plvi-frontend-mi355x 0.1 (gfx950)"; }

extern "C" int plvi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int plvi_device_malloc(void** ptr, size_t bytes) {
    if (!ptr) return PLVI_E_BADARG;
    PLVI_CHECK(hipMalloc(ptr, bytes));
    return PLVI_OK;
}

extern "C" int plvi_device_free(void* ptr) {
    PLVI_CHECK(hipFree(ptr));
    return PLVI_OK;
}

extern "C" int plvi_memcpy(void* dst, const void* src, size_t bytes, int kind) {
    const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost
                                                                         : hipMemcpyDeviceToDevice;
    if (kind < 1 || kind > 3) return PLVI_E_BADARG;
    PLVI_CHECK(hipMemcpy(dst, src, bytes, k));
    return PLVI_OK;
}

extern "C" int plvi_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream) {
    const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost
                                                                         : hipMemcpyDeviceToDevice;
    if (kind < 1 || kind > 3) return PLVI_E_BADARG;
    PLVI_CHECK(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
    return PLVI_OK;
}

extern "C" int plvi_device_synchronize(void) {
    PLVI_CHECK(hipDeviceSynchronize());
    return PLVI_OK;
}
