// tools/calib/pmc_calib.hip -- PMC calibration kernels (diagnostic, not part of
// the product).  MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE / WRITE_SIZE
// are exact only for 16-B-per-lane streaming accesses; other widths must be
// calibrated on a known byte count in the same access pattern.  These kernels
// stream a buffer with the widths the ORB / LSD kernels use:
//   calib_dword_read   4 B per lane loads (contiguous 256 B per wave instruction), 1 word per wave written
//   calib_dword_copy   4 B per lane loads and stores
//   calib_byte_copy    1 B per lane loads and stores
//   calib_dwordx2_store 8 B per lane stores (no loads)
//   calib_dwordx4_store 16 B per lane stores (no loads; the LBD Sobel kernels' int4 stores)
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o ../lib/libplvi_calib.so pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void calib_dword_read(const uint32_t* __restrict__ s, uint32_t* __restrict__ d, size_t n) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= s[i];
    acc = __reduce_or_sync(0xffffffffffffffffull, acc);
    if (threadIdx.x % 64 == 0) d[(blockIdx.x * 256 + threadIdx.x) / 64] = acc;
}
__global__ __launch_bounds__(256) void calib_dword_copy(const uint32_t* __restrict__ s, uint32_t* __restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = s[i] + 1u;
}
__global__ __launch_bounds__(256) void calib_byte_copy(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = s[i] + 1;
}
__global__ __launch_bounds__(256) void calib_dwordx2_store(uint2* __restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        d[i] = make_uint2((unsigned)i, (unsigned)(i >> 32));
}

__global__ __launch_bounds__(256) void calib_dwordx4_store(uint4* __restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        d[i] = make_uint4((unsigned)i, (unsigned)(i >> 32), 1u, 2u);
}

// mode 0..4 as listed above; n = bytes read (modes 0-2) or written (modes 3-4)
extern "C" int calib_run(int mode, const void* src, void* dst, size_t n, void* stream) {
    const dim3 g(4096), b(256);
    hipStream_t st = (hipStream_t)stream;
    if (mode == 0) hipLaunchKernelGGL(calib_dword_read, g, b, 0, st, (const uint32_t*)src, (uint32_t*)dst, n / 4);
    else if (mode == 1) hipLaunchKernelGGL(calib_dword_copy, g, b, 0, st, (const uint32_t*)src, (uint32_t*)dst, n / 4);
    else if (mode == 2) hipLaunchKernelGGL(calib_byte_copy, g, b, 0, st, (const uint8_t*)src, (uint8_t*)dst, n);
    else if (mode == 3) hipLaunchKernelGGL(calib_dwordx2_store, g, b, 0, st, (uint2*)dst, n / 8);
    else if (mode == 4) hipLaunchKernelGGL(calib_dwordx4_store, g, b, 0, st, (uint4*)dst, n / 16);
    else return 1;
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
