// FETCH_SIZE calibration for the load widths the search kernel issues
// (MI355X_MICROARCH.md 'HBM': only 16-B/lane streaming reads are calibrated).
// Each kernel streams the same 2 GiB buffer once with W-byte loads per lane in
// whole-wave contiguous runs (as eval_rows / eval_rows_h16 read a row) and the
// rocprofv3 --pmc FETCH_SIZE per dispatch is compared with 2 GiB.
// Build: hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <class T>
__global__ __launch_bounds__(256) void k_stream(const T* __restrict__ p, size_t n, float* out) {
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
        for (unsigned j = 0; j < sizeof(T) / 4; ++j) acc += __uint_as_float(w[j]);
    }
    if (acc == 1234.5f) out[blockIdx.x] = acc;  // keeps the loads live, never true for the zero buffer
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    void* buf = nullptr;
    float* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
    if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
    const int grid = 4096;
    hipLaunchKernelGGL(k_stream<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_stream<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_stream<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("streamed %zu bytes per kernel (widths 4, 8, 16 B/lane)\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
