// copy_roof.hip -- the device-to-device copy ceiling the edit kernels are compared
// with ("also report a measured device-to-device copy ceiling").
// A grid-stride 16-byte-per-lane copy kernel and hipMemcpyDtoD over the same byte
// counts as the bench workloads (read + write bytes = 2 x size).  Diagnostic tool.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void __launch_bounds__(256) copy16(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

// each wave copies whole 6 KiB tiles, 6 x 16 B per lane, like the wave lane's loads and stores
__global__ void __launch_bounds__(256) copy_tiles(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const size_t tiles = n / 384;
    for (size_t t = wave; t < tiles; t += waves) {
        uint4 v[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] = in[t * 384 + lane + 64 * k];
#pragma unroll
        for (int k = 0; k < 6; ++k) out[t * 384 + lane + 64 * k] = v[k];
    }
}

int main(int argc, char **argv) {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t sizes[] = {80000000ull, 1530000000ull, 3700000000ull};
    for (size_t sz : sizes) {
        const size_t n = sz / 16;
        uint4 *a, *b;
        if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&b, n * 16) != hipSuccess) return 1;
        hipMemset(a, 1, n * 16);
        hipMemset(b, 0, n * 16);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int iters = sz > 1000000000ull ? 20 : 200;
        struct {
            const char *name;
            int kind;
            int grid;
        } runs[] = {{"copy16 grid=CUs*8", 0, cus * 8}, {"copy16 grid=CUs*32", 0, cus * 32},
                    {"copy_tiles grid=CUs*4", 1, cus * 4}, {"hipMemcpyDtoD", 2, 0}};
        for (auto &r : runs) {
            for (int w = 0; w < 3; ++w) {
                if (r.kind == 0) hipLaunchKernelGGL(copy16, dim3(r.grid), dim3(256), 0, 0, a, b, n);
                else if (r.kind == 1) hipLaunchKernelGGL(copy_tiles, dim3(r.grid), dim3(256), 0, 0, a, b, n);
                else hipMemcpyAsync(b, a, n * 16, hipMemcpyDeviceToDevice, 0);
            }
            hipEventRecord(e0, 0);
            for (int i = 0; i < iters; ++i) {
                if (r.kind == 0) hipLaunchKernelGGL(copy16, dim3(r.grid), dim3(256), 0, 0, a, b, n);
                else if (r.kind == 1) hipLaunchKernelGGL(copy_tiles, dim3(r.grid), dim3(256), 0, 0, a, b, n);
                else hipMemcpyAsync(b, a, n * 16, hipMemcpyDeviceToDevice, 0);
            }
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double per = ms / iters;
            printf("copy %10zu B  %-24s %9.1f us  %7.1f GB/s (read+write)\n", sz, r.name, per * 1e3,
                   2.0 * sz / (per * 1e-3) / 1e9);
        }
        hipFree(a);
        hipFree(b);
    }
    return 0;
}
