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

// An SALU write of EXEC directly before a DPP op: the shape of the first wk_store_mtu's
// pass-2 read (the s_or_b64 exec that ends the pass-1 store branches, then v_mov_b32_dpp
// ... wave_shr:1).  Here in one asm block: EXEC to `part`, a VALU op under it, EXEC back to
// the full mask, NOPS wait states, the DPP shift.
#define DPP_EXEC_SEQ(NOPSTR)                                                                     \
    asm volatile("s_mov_b64 %[sv], exec\n\t"                                                   \
                 "s_mov_b64 exec, %[pt]\n\t"                                                   \
                 "v_mov_b32 %[o], 0\n\t"                                                       \
                 "s_mov_b64 exec, %[sv]\n\t" NOPSTR                                            \
                 "v_mov_b32_dpp %[o], %[v] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"  \
                 : [o] "=&v"(o), [sv] "=&s"(saved)                                               \
                 : [v] "v"(v), [pt] "s"(part))

// out: [no wait states, 5 wait states, wave_prev after a divergent branch's join, the bare
// DPP builtin after one, (scratch)] x 64
__global__ __launch_bounds__(64) void dpp_exec_kernel(const uint32_t *in, uint64_t part, uint32_t *out) {
    const int lane = threadIdx.x;
    const uint32_t v = in[lane];
    uint32_t o;
    uint64_t saved;
    DPP_EXEC_SEQ("");
    out[lane] = o;
    DPP_EXEC_SEQ("s_nop 4\n\t");
    out[64 + lane] = o;
    // the product's helper right after a divergent branch (the compiler's own EXEC restore)
    if ((part >> lane) & 1ull) out[256 + lane] = v * 3u + 1u;
    out[128 + lane] = wave_prev(v);
    // ... and the bare builtin in the same place
    if ((part >> lane) & 1ull) out[256 + lane] = v * 5u + 1u;
    out[192 + lane] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}

extern "C" int dpp_exec_run(const uint32_t *h_in, uint64_t part, uint32_t *h_out) {
    uint32_t *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc((void **)&d_in, 64 * 4) != hipSuccess || hipMalloc((void **)&d_out, 5 * 64 * 4) != hipSuccess)
        return -1;
    int rc = 0;
    if (hipMemcpy(d_in, h_in, 64 * 4, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(dpp_exec_kernel, dim3(1), dim3(64), 0, 0, d_in, part, d_out);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(h_out, d_out, 5 * 64 * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = -1;
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
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
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}

// DPP folded into a VOP2 op (the compiler's DPP combine): wave_shr:1 on src0 of v_subrev /
// v_sub / v_add / v_max, and v_subrev with row_shr:1, against b - prev(a) etc. -- the first
// wk_store_mtu's second pass-2 read was `v_subrev_u32_dpp v2, v78, v2 wave_shr:1`.
// out: [subrev, sub, add, max, subrev row_shr:1, or, lshlrev] x 64
#define DPP_VOP2(OP, CTRL, dst, a, b)                                                          \
    asm volatile(OP "_dpp %0, %1, %2 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1"        \
                 : "=&v"(dst) : "v"(a), "v"(b))
__global__ __launch_bounds__(64) void dpp_vop2_kernel(const uint32_t *in, uint32_t *out) {
    const int lane = threadIdx.x;
    const uint32_t a = in[lane], b = 1000000u + 1000u * (uint32_t)lane;
    uint32_t r0, r1, r2, r3, r4, r5, r6;
    DPP_VOP2("v_subrev_u32", "wave_shr:1", r0, a, b);
    DPP_VOP2("v_sub_u32", "wave_shr:1", r1, a, b);
    DPP_VOP2("v_add_u32", "wave_shr:1", r2, a, b);
    DPP_VOP2("v_max_u32", "wave_shr:1", r3, a, b);
    DPP_VOP2("v_subrev_u32", "row_shr:1", r4, a, b);
    DPP_VOP2("v_or_b32", "wave_shr:1", r5, a, b);
    DPP_VOP2("v_lshlrev_b32", "wave_shr:1", r6, a, b);
    out[lane] = r0;
    out[64 + lane] = r1;
    out[128 + lane] = r2;
    out[192 + lane] = r3;
    out[256 + lane] = r4;
    out[320 + lane] = r5;
    out[384 + lane] = r6;
}

extern "C" int dpp_vop2_run(const uint32_t *h_in, uint32_t *h_out) {
    uint32_t *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc((void **)&d_in, 64 * 4) != hipSuccess || hipMalloc((void **)&d_out, 7 * 64 * 4) != hipSuccess)
        return -1;
    int rc = 0;
    if (hipMemcpy(d_in, h_in, 64 * 4, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(dpp_vop2_kernel, dim3(1), dim3(64), 0, 0, d_in, d_out);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(h_out, d_out, 7 * 64 * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = -1;
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}
