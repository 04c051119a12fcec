// capi.hip — library-level entry points of the C-ABI (include/plvi_frontend.h).
#include <hip/hip_runtime.h>

#include "plvi_common.h"

extern "C" const char* plvi_version(void) { return "plvi-frontend-mi355x 0.1 (gfx950)"; }

extern "C" int plvi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
