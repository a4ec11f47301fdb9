// tcpreplay_kernels.hip -- tcpreplay's file-output pass with --unique-ip on gfx950.
//
// One pass of send_packets (src/send_packets.c:379-646) over a device-resident capture,
// as `tcpreplay -w` writes it (sendpacket.c:485-486, 945-968):
//   tr_mark   one thread per record: fast_edit_packet (send_packets.c:124-257) -- the
//             source / destination address shifted by the pass's iteration in a way that
//             keeps the checksums (no checksum is touched) -- or, under -K (preload), the
//             cached record edited in place by one step; the record's output size (0 when
//             the edit fails: the reference counts it failed and does not send it)
//   scan      exclusive sum of the sizes (hipCUB) -> output offsets
//   tr_write  one wave per record: the record header (timestamp fraction as libpcap's
//             nanosecond read leaves it) and the bytes, the new addresses patched in
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "edit_pkt.hpp"
#include "tcpreplay_hip_dev.h"

namespace {
using te::u8;
using te::u32;

__device__ __forceinline__ u32 rd32(const u8 *p, bool sw) {
    const u32 v = (u32)p[0] | (u32)p[1] << 8 | (u32)p[2] << 16 | (u32)p[3] << 24;
    return sw ? __builtin_bswap32(v) : v;
}
__device__ __forceinline__ u32 be32at(const u8 *p) {
    return (u32)p[0] << 24 | (u32)p[1] << 16 | (u32)p[2] << 8 | (u32)p[3];
}

// fast_edit_packet: the new source / destination (host order) and where they go, or -1
// a record's caplen as get_next_packet returns it: safe_pcap_next (send_packets.c:955,985 ->
// src/common/utils.c:159-162) trims it to len (the host walk stopped at a zero len or caplen)
__device__ __forceinline__ u32 rd_cap(const u8 *rec, bool sw) {
    const u32 cl = rd32(rec + 8, sw), pl = rd32(rec + 12, sw);
    return pl < cl ? pl : cl;
}

__device__ int fast_edit(const u8 *pkt, u32 caplen, uint64_t iteration, bool cached, u32 &src, u32 &dst,
                         u32 &at_s, u32 &at_d) {
    te::L2 r;
    if (te::get_l2len_protocol(pkt, caplen, r) < 0) return -1;
    if (r.protocol == 0x0800) {
        if (caplen < r.l2len + 20) return -1;
        at_s = r.l2len + 12;
        at_d = r.l2len + 16;
    } else if (r.protocol == 0x86DD) {
        if (caplen < r.l2len + 40) return -1;
        at_s = r.l2len + 8 + 12;  // ip_src.__u6_addr32[3]
        at_d = r.l2len + 24 + 12;
    } else {
        return -1;
    }
    const u32 so = be32at(pkt + at_s), dor = be32at(pkt + at_d);
    src = so;
    dst = dor;
    // COUNTER (64-bit) arithmetic in the cached compare, as the reference's types give it
    if ((!cached && dst > src) || (cached && ((uint64_t)dst - iteration) > ((uint64_t)src - 1 - iteration))) {
        if (cached) {
            --src;
            ++dst;
        } else {
            src -= (u32)iteration;
            dst += (u32)iteration;
        }
        if (src > so && dst > dor) --src;  // the wrap compensations (:180-205)
        else if (dst < dor && src < so) ++dst;
    } else {
        if (cached) {
            ++src;
            --dst;
        } else {
            src += (u32)iteration;
            dst -= (u32)iteration;
        }
        if (dst > dor && src > so) --dst;
        else if (src < so && dst < dor) ++src;
    }
    return 0;
}

// check_list (src/common/list.c:139-156) and send_packets.c:440-447's rule: true when the
// include / exclude list leaves packet `v` (1-based within the pass) out
__device__ __forceinline__ bool listed_out(const uint64_t *l, uint32_t n, bool exclude, uint64_t v) {
    bool set = false;
    for (uint32_t i = 0; i < n && !set; ++i) {
        const uint64_t mn = l[2 * i], mx = l[2 * i + 1];
        set = (mn != 0 && mx != 0) ? (v >= mn && v <= mx) : (mn == 0 ? v <= mx : v >= mn);
    }
    return set == exclude;
}

__global__ __launch_bounds__(256) void tr_mark(TrPass a) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const uint64_t off = a.off[j];
    const u8 *rec = (a.cache ? a.cache : a.img) + off;
    const u32 caplen = rd_cap(rec, a.swapped != 0);
    u32 keep = 1, at_s = 0, src = 0, dst = 0, at_d = 0;
    if (a.list && listed_out(a.list, a.nlist, a.exclude != 0, j + 1)) {
        keep = 0;  // skipped before anything else: not edited, not sent, not counted failed
    } else if (a.edit) {
        if (fast_edit(rec + 16, caplen, a.iteration, a.cached != 0, src, dst, at_s, at_d) < 0) {
            keep = 0;
            if (a.nfail) atomicAdd((unsigned long long *)a.nfail, 1ull);
        } else if (a.cache) {  // -K: the cached record itself (the next pass starts from it)
            u8 *p = a.cache + off + 16;
            for (int k = 0; k < 4; ++k) {
                p[at_s + k] = (u8)(src >> (24 - 8 * k));
                p[at_d + k] = (u8)(dst >> (24 - 8 * k));
            }
            at_s = 0;
        }
    }
    a.size[j] = keep ? 16ull + caplen : 0ull;
    ((uint4 *)a.patch)[j] = make_uint4(at_s, src, at_d, dst);  // at_s 0: nothing to patch (offsets are >= 20)
}

// one wave per record: header + bytes (loads of a record by 64 consecutive lanes)
__global__ __launch_bounds__(256) void tr_write(TrPass a) {
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= a.n || a.size[j] == 0) return;
    const u8 *rec = (a.cache ? a.cache : a.img) + a.off[j];
    u8 *o = a.out + a.pos[j];
    const bool sw = a.swapped != 0;
    const u32 caplen = rd_cap(rec, sw);
    if (lane < 4) {  // ts_sec, the fraction (x1000 for a microsecond capture), caplen, len
        u32 v = lane == 2 ? caplen : rd32(rec + 4 * lane, sw);
        if (lane == 1 && !a.nsec) v *= 1000u;
        for (int k = 0; k < 4; ++k) o[4 * lane + k] = (u8)(v >> (8 * k));
    }
    const uint4 pt = ((const uint4 *)a.patch)[j];
    for (u32 i = lane; i < caplen; i += 64) {
        u8 b = rec[16 + i];
        if (pt.x) {
            if (i - pt.x < 4) b = (u8)(pt.y >> (24 - 8 * (i - pt.x)));
            else if (i - pt.z < 4) b = (u8)(pt.w >> (24 - 8 * (i - pt.z)));
        }
        o[16 + i] = b;
    }
}

// one thread per cache byte (4 records): 11 (send, C2S) unless the list leaves it out (00)
__global__ __launch_bounds__(256) void tr_dirbits(const uint64_t *l, uint32_t nl, int32_t exclude, uint64_t n,
                                                  u8 *bits) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= (n + 3) / 4) return;
    u32 v = 0;
    for (int k = 0; k < 4; ++k) {
        const uint64_t j = 4 * b + k;
        if (j < n && !listed_out(l, nl, exclude != 0, j + 1)) v |= 3u << (2 * k);
    }
    bits[b] = (u8)v;
}
}  // namespace

extern "C" int tr_list_dirbits(const uint64_t *d_list, uint32_t nlist, int exclude, uint64_t n, uint8_t *d_bits,
                               void *stream) {
    if (n == 0) return 0;
    const uint64_t nb = (n + 3) / 4;
    if (nb > 0xffffffffull * 256) return -1;
    hipLaunchKernelGGL(tr_dirbits, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_list,
                       nlist, exclude, n, d_bits);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" size_t tr_scan_temp_bytes(uint64_t n) {
    size_t t = 0;
    const hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const unsigned long long *)nullptr,
                                                          (unsigned long long *)nullptr, (int)n);
    return e == hipSuccess ? t : 0;
}

extern "C" int tr_launch_pass(const TrPass *p, void *temp, size_t temp_bytes, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (p->n == 0) return 0;
    if (p->n > 0x7fffffffull) return -1;
    TrPass a = *p;
    hipLaunchKernelGGL(tr_mark, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
    if (a.mark_only) return hipGetLastError() == hipSuccess ? 0 : -1;
    size_t tb = temp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(temp, tb, (const unsigned long long *)a.size, (unsigned long long *)a.pos,
                                         (int)a.n, st) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(tr_write, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
