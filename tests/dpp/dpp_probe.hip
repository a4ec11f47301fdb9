// dpp_probe.hip -- TEST INFRASTRUCTURE: the product's wave_dpp.hpp helpers (wave_prev,
// wave_scan_add, wave_scan_max, wave_or) run by one wave under full EXEC and under a
// divergent EXEC mask, with the LDS shift the helpers replace computed alongside by the same
// lanes (tests/test_dpp.py compares them).  Built into tests/dpp/_build/libdppprobe.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_dpp.hpp"

// out: [prev, add, max, or, lds_prev] x 64
__global__ __launch_bounds__(64) void dpp_probe_kernel(const uint32_t *in, uint64_t mask, int divergent, uint32_t *out) {
    __shared__ uint32_t lds[64];
    const int lane = threadIdx.x;
    const uint32_t v = in[lane];
    lds[lane] = v;
    __syncthreads();
    uint32_t p = 0xdeadbeefu, a = 0xdeadbeefu, m = 0xdeadbeefu, o = 0xdeadbeefu, l = 0xdeadbeefu;
    if (!divergent) {
        p = wave_prev(v);
        a = wave_scan_add(v);
        m = wave_scan_max(v);
        o = wave_or(v);
        l = lane ? lds[lane - 1] : 0u;
    } else if ((mask >> lane) & 1ull) {  // these lanes only: the others are off in EXEC
        p = wave_prev(v);
        a = wave_scan_add(v);
        m = wave_scan_max(v);
        o = wave_or(v);
        l = lane ? lds[lane - 1] : 0u;
    }
    out[lane] = p;
    out[64 + lane] = a;
    out[128 + lane] = m;
    out[192 + lane] = o;
    out[256 + lane] = l;
}

extern "C" int dpp_probe_run(const uint32_t *h_in, uint64_t mask, int divergent, uint32_t *h_out) {
    uint32_t *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc((void **)&d_in, 64 * 4) != hipSuccess || hipMalloc((void **)&d_out, 5 * 64 * 4) != hipSuccess)
        return -1;
    int rc = 0;
    if (hipMemcpy(d_in, h_in, 64 * 4, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(dpp_probe_kernel, dim3(1), dim3(64), 0, 0, d_in, mask, divergent, d_out);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(h_out, d_out, 5 * 64 * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = -1;
    }
    hipFree(d_in);
    hipFree(d_out);
    return rc;
}
