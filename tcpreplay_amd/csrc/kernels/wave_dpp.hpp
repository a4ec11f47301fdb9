// wave_dpp.hpp -- cross-lane steps of one wave in VALU with GFX9 DPP (gfx950): OR and
// inclusive add / max scans over the 64 lanes, and the previous lane's value.  DPP row
// shifts work within each 16-lane row; row_bcast:15 / row_bcast:31 carry the rows' totals
// on, wave_shr:1 shifts the whole wave by one lane (__shfl_up and friends would be
// ds_bpermute round trips through the LDS pipe).
//
// Call these where every lane of the wave is active (wave-uniform control flow).  A DPP
// operand read from a lane that EXEC has switched off does not return that lane's value:
// with bound_ctrl (as here) it reads 0.  A DPP op right behind the SALU write of EXEC that
// ends a divergent branch reads the lanes the new EXEC has on (no wait states needed).
//
// The product builds with the compiler's DPP combine off (-mllvm -amdgpu-dpp-combine=false,
// tcpreplay_amd/csrc/Makefile): the combine folds a DPP mov into the VALU op that uses it,
// and on MI355X a folded "reversed" VOP2 op applies the DPP lane pattern to src1 instead of
// src0 -- v_subrev_u32_dpp d, a, b wave_shr:1 gives prev(b) - a, not b - prev(a), and
// v_lshlrev_b32_dpp likewise (tests/test_dpp.py, the probe kernels in tests/dpp/).  That was
// the first wk_store_mtu's wrong output: its pass-2 `q - pop` with pop = wave_prev(my_op)
// became v_subrev_u32_dpp, and the chunks took their first bytes from the wrong place.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// OR over the wave: each row's OR gathers in its lane 15, four readlanes combine the rows
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    return (uint32_t)(__builtin_amdgcn_readlane((int)v, 15) | __builtin_amdgcn_readlane((int)v, 31) |
                      __builtin_amdgcn_readlane((int)v, 47) | __builtin_amdgcn_readlane((int)v, 63));
}

// inclusive scans: row_shr 1/2/4/8 scan each 16-lane row, row_bcast:15 (rows 1 and 3) and
// row_bcast:31 (rows 2 and 3) add the earlier rows' totals; lanes a row mask leaves out
// take `old` = 0, the identity of both operations
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
// the previous lane's value (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t wave_prev(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}
