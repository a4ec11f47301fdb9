// lds_probe.hip -- diagnostic: (1) does ds_read_b128 / ds_read_b64 at a 4-byte aligned (not
// 16-byte aligned) LDS address return the 16 bytes there on this box (the alignment mode the
// driver sets), and (2) the cost of reading an 84-byte window per lane at an 80-byte lane
// stride (C2's record stride) as 21 dwords (ds_read2_b32 pairs) vs 6 unaligned ds_read_b128.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint4 lds_b128(const uint8_t *p) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
    return v;
}
__device__ __forceinline__ uint2 lds_b64(const uint8_t *p) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
    return v;
}

__global__ void probe_align(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t S[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) S[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const int lane = threadIdx.x;
    const uint32_t off = 4u * (uint32_t)lane;  // 4-byte aligned, every residue mod 16
    const uint4 v = lds_b128(S + off);
    const uint2 w = lds_b64(S + off);
    const uint32_t *q = (const uint32_t *)(S + off);
    out[lane] = (v.x == q[0] && v.y == q[1] && v.z == q[2] && v.w == q[3]) ? 1u : 0u;
    out[64 + lane] = (w.x == q[0] && w.y == q[1]) ? 1u : 0u;
}

// windows at an 80-byte stride: 21 dwords (the compiler's ds_read2_b32) vs 6 x b128
template <int MODE>
__global__ void __launch_bounds__(256) win_reads(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t S[4][64 * 80 + 256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * (64 * 80 + 256) / 4; i += 256) ((uint32_t *)S)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t base = 80u * (uint32_t)lane + 16u + 4u * (uint32_t)((it + lane) & 0);  // dword aligned
        const uint8_t *p = S[w] + base + 12u;  // packet start - 2, rounded: 4-byte aligned, 12 mod 16
        if (MODE == 0) {
            const uint32_t *d = (const uint32_t *)p;
#pragma unroll
            for (int j = 0; j < 21; ++j) acc += d[j] ^ (uint32_t)j;
        } else {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                uint4 v;
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"((uint32_t)(uintptr_t)p), "i"(16 * j));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                acc += v.x ^ v.y ^ v.z ^ v.w;
            }
        }
        asm volatile("" : "+v"(acc));
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
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
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(win_reads<0>, dim3(1024), dim3(256), 0, 0, d, 200);
            else hipLaunchKernelGGL(win_reads<1>, dim3(1024), dim3(256), 0, 0, d, 200);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) printf("window reads mode %d (%s): %.3f ms\n", mode, mode ? "6 x b128" : "21 dwords", ms);
        }
    }
    return 0;
}
