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

extern "C" int plvi_stream_create(void** stream) {
    if (!stream) return PLVI_E_BADARG;
    hipStream_t s = nullptr;
    PLVI_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void*)s;
    return PLVI_OK;
}

extern "C" int plvi_stream_destroy(void* stream) {
    if (!stream) return PLVI_E_BADARG;
    PLVI_CHECK(hipStreamDestroy((hipStream_t)stream));
    return PLVI_OK;
}

extern "C" int plvi_stream_synchronize(void* stream) {
    PLVI_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return PLVI_OK;
}

extern "C" int plvi_event_create(void** event) {
    if (!event) return PLVI_E_BADARG;
    hipEvent_t e = nullptr;
    PLVI_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *event = (void*)e;
    return PLVI_OK;
}

extern "C" int plvi_event_record(void* event, void* stream) {
    if (!event) return PLVI_E_BADARG;
    PLVI_CHECK(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return PLVI_OK;
}

extern "C" int plvi_stream_wait_event(void* stream, void* event) {
    if (!event) return PLVI_E_BADARG;
    PLVI_CHECK(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
    return PLVI_OK;
}

extern "C" int plvi_event_destroy(void* event) {
    if (!event) return PLVI_E_BADARG;
    PLVI_CHECK(hipEventDestroy((hipEvent_t)event));
    return PLVI_OK;
}

// HIP graphs: a batch step (any sequence of plvi_* calls on `stream`, their
// internal streams joined by events) captured once and replayed with one
// launch, which takes the per-call host work (~100 API calls per frame
// schedule) off the path of small batches.
extern "C" int plvi_graph_capture_begin(void* stream) {
    if (!stream) return PLVI_E_BADARG;  // the legacy null stream cannot be captured
    PLVI_CHECK(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeRelaxed));
    return PLVI_OK;
}

extern "C" int plvi_graph_capture_end(void* stream, void** graph_exec) {
    if (!stream || !graph_exec) return PLVI_E_BADARG;
    hipGraph_t g = nullptr;
    PLVI_CHECK(hipStreamEndCapture((hipStream_t)stream, &g));
    hipGraphExec_t e = nullptr;
    const hipError_t rc = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (rc != hipSuccess) return PLVI_E_HIP;
    *graph_exec = (void*)e;
    return PLVI_OK;
}

extern "C" int plvi_graph_launch(void* graph_exec, void* stream) {
    if (!graph_exec) return PLVI_E_BADARG;
    PLVI_CHECK(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream));
    return PLVI_OK;
}

extern "C" int plvi_graph_destroy(void* graph_exec) {
    if (graph_exec) PLVI_CHECK(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
    return PLVI_OK;
}
