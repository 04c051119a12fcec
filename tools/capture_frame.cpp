// Diagnostic: capture plvi_frame_extract_batch (the multi-stream frame
// schedule, lines_pipeline.hip run_with_orb) into a HIP graph through the
// C-ABI, with a SIGSEGV handler that prints the host backtrace of the crash.
// usage: capture_frame [n_frames] [warm 0|1] [mode 0=relaxed 1=global 2=thread-local]
// Built by tools/build_capture.sh against lib/libplvi_frontend.so.
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "plvi_frontend.h"

static void on_segv(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "\n*** SIGSEGV, host backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    _exit(128 + sig);
}

#define CK(x)                                                                 \
    do {                                                                      \
        int e_ = (int)(x);                                                    \
        if (e_) {                                                             \
            printf("  %s -> %d (line %d)\n", #x, e_, __LINE__);               \
            fflush(stdout);                                                   \
            return 1;                                                         \
        }                                                                     \
    } while (0)

int main(int argc, char** argv) {
    signal(SIGSEGV, on_segv);
    const int n = argc > 1 ? atoi(argv[1]) : 16;
    const int warm = argc > 2 ? atoi(argv[2]) : 1;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const int W = 640, H = 480;
    std::vector<uint8_t> host((size_t)n * W * H);
    unsigned s = 12345u;
    for (auto& b : host) {
        s = s * 1664525u + 1013904223u;
        b = (uint8_t)(s >> 24);
    }
    uint8_t* d = nullptr;
    CK(hipMalloc(&d, host.size()));
    CK(hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice));
    plvi_orb_params op = {1000, 1.2f, 8, 20, 7, 0};
    plvi_line_params lp = {200, 0, 0.8f, 2, 2.0f, 0, 0};
    plvi_orb_extractor* orb = nullptr;
    plvi_line_extractor* lx = nullptr;
    CK(plvi_orb_create(&op, W, H, n, 0, &orb));
    CK(plvi_lines_create(&lp, W, H, n, 0, &lx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (warm) {
        CK(plvi_frame_extract_batch(orb, lx, d, n, (size_t)W * H, W, 0, 0, st));
        CK(hipStreamSynchronize(st));
        printf("direct ok\n");
        fflush(stdout);
    }
    const hipStreamCaptureMode m = mode == 1 ? hipStreamCaptureModeGlobal
                                   : mode == 2 ? hipStreamCaptureModeThreadLocal
                                               : hipStreamCaptureModeRelaxed;
    CK(hipStreamBeginCapture(st, m));
    printf("capturing\n");
    fflush(stdout);
    const int rc = plvi_frame_extract_batch(orb, lx, d, n, (size_t)W * H, W, 0, 0, st);
    printf("schedule issued rc=%d\n", rc);
    fflush(stdout);
    hipStreamCaptureStatus cs;
    CK(hipStreamIsCapturing(st, &cs));
    printf("capture status %d\n", (int)cs);
    fflush(stdout);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(st, &g);
    printf("end capture -> %s\n", hipGetErrorString(e));
    fflush(stdout);
    if (e != hipSuccess) return 1;
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    printf("graph nodes %zu\n", nn);
    hipGraphExec_t ge = nullptr;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    printf("replay ok\n");
    return 0;
}
