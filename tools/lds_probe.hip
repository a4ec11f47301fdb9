// lds_probe.hip -- diagnostic: (1) does ds_read_b128 / ds_read_b64 at a 4-byte aligned (not
// 16-byte aligned) LDS address return the bytes there on this box (the driver's alignment
// mode), and (2) the LDS cost of two read patterns of the wave lane, timed over many
// iterations (reads of one batch in flight together, one wait a batch):
//   chunk: 16 bytes a lane at a 16-byte lane stride, 4 bytes off 16-byte alignment (the
//          sized store's shifted chunks): 4 x ds_read_b32 | 1 unaligned ds_read_b128 |
//          2 aligned ds_read_b128 + dword selects
//   window: 84 bytes a lane at an 80-byte lane stride (C2's records): 21 dwords as the
//          compiler reads them | 6 unaligned ds_read_b128
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint4 b128(uint32_t a) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__global__ void probe_align(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t S[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) S[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const int lane = threadIdx.x;
    const uint32_t off = 4u * (uint32_t)lane;
    const uint4 v = b128((uint32_t)(uintptr_t)(S + off));
    uint2 w;
    asm volatile("ds_read_b64 %0, %1" : "=v"(w) : "v"((uint32_t)(uintptr_t)(S + off)));
    wait_lds();
    const uint32_t *q = (const uint32_t *)(S + off);
    out[lane] = (v.x == q[0] && v.y == q[1] && v.z == q[2] && v.w == q[3]) ? 1u : 0u;
    out[64 + lane] = (w.x == q[0] && w.y == q[1]) ? 1u : 0u;
}

template <int MODE>
__global__ void __launch_bounds__(256) chunk_reads(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t S[4][8 * 1024 + 64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * (8 * 1024 + 64) / 4; i += 256) ((uint32_t *)S)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    const uint32_t base = (uint32_t)(uintptr_t)S[w];
    for (int it = 0; it < iters; ++it) {
        const uint32_t sh = 4u * (uint32_t)((it >> 2) & 3);  // the shift: wave-uniform here
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t *d = (const uint32_t *)(S[w] + 16u * ((uint32_t)lane + 64u * k) + sh);
                acc += d[0] ^ d[1] ^ d[2] ^ d[3];
            }
        } else if (MODE == 1) {
            uint4 v[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) v[k] = b128(base + 16u * ((uint32_t)lane + 64u * k) + sh);
            wait_lds();
#pragma unroll
            for (int k = 0; k < 6; ++k) acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        } else {
            uint4 p[6], q[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t a = (base + 16u * ((uint32_t)lane + 64u * k) + sh) & ~15u;
                p[k] = b128(a);
                q[k] = b128(a + 16u);
            }
            wait_lds();
            const uint32_t s = sh >> 2;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t x[8] = {p[k].x, p[k].y, p[k].z, p[k].w, q[k].x, q[k].y, q[k].z, q[k].w};
                uint32_t r = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) r ^= s == 0 ? x[i] : s == 1 ? x[i + 1] : s == 2 ? x[i + 2] : x[i + 3];
                acc += r;
            }
        }
        asm volatile("" : "+v"(acc));
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
__global__ void __launch_bounds__(256) win_reads(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t S[4][64 * 80 + 256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * (64 * 80 + 256) / 4; i += 256) ((uint32_t *)S)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t a = (uint32_t)(uintptr_t)S[w] + 80u * (uint32_t)lane + 28u;  // packet - 2, 4-aligned
        if (MODE == 0) {
            const uint32_t *d = (const uint32_t *)(S[w] + 80u * (uint32_t)lane + 28u);
#pragma unroll
            for (int j = 0; j < 21; ++j) acc += d[j] ^ (uint32_t)j;
        } else {
            uint4 v[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) v[j] = b128(a + 16u * j);
            wait_lds();
#pragma unroll
            for (int j = 0; j < 6; ++j) acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        }
        asm volatile("" : "+v"(acc));
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename K>
static float timeit(K k, uint32_t *d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0;
    int it = 400;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        void *args[] = {&d, &it};
        const hipError_t e = hipLaunchKernel((const void *)k, dim3(1024), dim3(256), args, 0, 0);
        if (e != hipSuccess) printf("launch: %s\n", hipGetErrorString(e));
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const hipError_t e2 = hipDeviceSynchronize();
    if (e2 != hipSuccess) printf("sync: %s\n", hipGetErrorString(e2));
    return ms;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 4 << 20);
    hipLaunchKernelGGL(probe_align, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[128];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int ok128 = 0, ok64 = 0;
    for (int i = 0; i < 64; ++i) ok128 += h[i], ok64 += h[64 + i];
    printf("unaligned ds_read_b128 correct lanes %d/64, ds_read_b64 %d/64\n", ok128, ok64);
    printf("chunk 4 x b32:           %.3f ms\n", timeit(chunk_reads<0>, d));
    printf("chunk unaligned b128:    %.3f ms\n", timeit(chunk_reads<1>, d));
    printf("chunk 2 aligned b128+sel %.3f ms\n", timeit(chunk_reads<2>, d));
    printf("window 21 dwords:        %.3f ms\n", timeit(win_reads<0>, d));
    printf("window 6 unaligned b128: %.3f ms\n", timeit(win_reads<1>, d));
    return 0;
}
