// Diagnostic: which fork/join pattern makes hipStreamEndCapture fail?
// Mirrors LinePipeline::run_with_orb (lines_pipeline.hip): the origin stream
// forks to `crit` (and crit2) and two aux streams through events, work runs
// on each, and everything joins back before the capture ends.
// usage: capture_probe <variant>
//   0: plain non-blocking streams, fresh events
//   1: priority streams (greatest / least), fresh events
//   2: as 1, events first used outside a capture (the bench's warm-up)
//   3: as 2, relaxed capture mode
//   4: as 3 with a fork event recorded twice (reuse inside one capture)
//   5: as 3, a stream that waits on an event recorded on a NON-captured stream
//   6: as 3, hipSetDevice + hipGetLastError between the captured calls
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_add(int* p, int v) {
    if (threadIdx.x == 0) atomicAdd(p, v);
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("  %s -> %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);          \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

static int schedule(hipStream_t st, hipStream_t crit, hipStream_t a0, hipStream_t a1, hipEvent_t* ev, int* d,
                    int variant, hipStream_t outside) {
    if (variant == 6) CK(hipSetDevice(0));
    CK(hipEventRecord(ev[0], st));                 // fork
    CK(hipStreamWaitEvent(crit, ev[0], 0));
    if (variant == 6) {
        CK(hipSetDevice(0));
        CK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, crit, d, 1);  // prep
    CK(hipEventRecord(ev[1], crit));               // evPrep
    CK(hipStreamWaitEvent(a0, variant == 4 ? ev[1] : ev[0], 0));
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, a0, d, 10);  // ORB
    CK(hipEventRecord(ev[2], a0));                 // evOrb
    CK(hipEventRecord(ev[3], crit));               // evGate
    if (variant == 5) CK(hipStreamWaitEvent(a1, ev[7], 0));  // recorded on `outside`
    CK(hipStreamWaitEvent(a1, ev[3], 0));
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, a1, d, 100);  // Sobel
    CK(hipEventRecord(ev[4], a1));                 // evSobel
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, crit, d, 1000);  // grow
    CK(hipStreamWaitEvent(crit, ev[4], 0));
    hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, crit, d, 10000);  // describe
    CK(hipEventRecord(ev[5], crit));               // evCrit
    CK(hipStreamWaitEvent(st, ev[5], 0));
    CK(hipStreamWaitEvent(st, ev[2], 0));
    if (variant == 4) {
        CK(hipEventRecord(ev[0], st));  // the fork event again, inside the same capture
        CK(hipStreamWaitEvent(crit, ev[0], 0));
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, crit, d, 100000);
        CK(hipEventRecord(ev[5], crit));
        CK(hipStreamWaitEvent(st, ev[5], 0));
    }
    (void)outside;
    return 0;
}

int main(int argc, char** argv) {
    const int variant = argc > 1 ? atoi(argv[1]) : 0;
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t st, crit, a0, a1, outside;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&outside, hipStreamNonBlocking));
    if (variant >= 1) {
        CK(hipStreamCreateWithPriority(&crit, hipStreamNonBlocking, greatest));
        CK(hipStreamCreateWithPriority(&a0, hipStreamNonBlocking, greatest));
        CK(hipStreamCreateWithPriority(&a1, hipStreamNonBlocking, least));
    } else {
        CK(hipStreamCreateWithFlags(&crit, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&a0, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&a1, hipStreamNonBlocking));
    }
    hipEvent_t ev[8];
    for (auto& evx : ev) CK(hipEventCreateWithFlags(&evx, hipEventDisableTiming));
    int* d = nullptr;
    CK(hipMalloc(&d, sizeof(int)));
    CK(hipMemset(d, 0, sizeof(int)));
    if (variant >= 2) {
        if (schedule(st, crit, a0, a1, ev, d, 0, outside)) return 1;
        CK(hipStreamSynchronize(st));
    }
    if (variant == 5) CK(hipEventRecord(ev[7], outside));
    printf("variant %d: begin capture\n", variant);
    fflush(stdout);
    CK(hipStreamBeginCapture(st, variant >= 3 ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal));
    if (schedule(st, crit, a0, a1, ev, d, variant, outside)) return 1;
    printf("variant %d: end capture\n", variant);
    fflush(stdout);
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(st, &g));
    hipGraphExec_t ge = nullptr;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipMemset(d, 0, sizeof(int)));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    int h = 0;
    CK(hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost));
    printf("variant %d: replay ok, sum %d\n", variant, h);
    return 0;
}
