// tcpedit_kernels.hip -- gfx950 kernels for the tcpedit rewrite path.
//
// One kernel, te_edit_tiles, runs the whole device pipeline of
// rewrite_packets() (src/tcprewrite.c:260-373) over a pcap image resident in
// HBM, in a single pass:
//   1. a block takes the next tile ticket (tiles = runs of consecutive records,
//      built from the record index so their LDS slots fit the block's budget);
//   2. the tile's byte span is streamed HBM -> LDS with 16-byte loads, each
//      record landing in its own slot whose alignment mod 16 equals its HBM
//      alignment (so every chunk is one aligned 16-byte LDS store);
//   3. one lane per packet runs tcpedit_packet() in LDS (edit_pkt.hpp);
//   4. a block scan of the output record sizes plus a decoupled look-back over
//      earlier tiles gives the tile's output offset (no second pass over HBM);
//   5. the block streams its output records LDS -> HBM as 16-byte chunks.
// Records too large for a tile are staged in an HBM scratch slot instead
// (same code, the slot pointer is in the global address space).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edit_pkt.hpp"
#include "te_kernels.h"

using namespace te;

namespace {

constexpr int BLOCK = TE_BLOCK;
constexpr int NWAVES = BLOCK / 64;

struct LaunchArgs {
    const te_dev_cfg_t *cfg;
    const uint16_t *portlut;
    const uint8_t *dirbits;   // tcpprep cache data (2 bits/packet) or null
    uint64_t dirbits_len;
    uint64_t pkt_base;        // packet number (0-based) of this run's first record
    int32_t fixed_dir;        // >= 0: caller-supplied direction (tcpedit_packet), NOSEND still edits
    const uint8_t *in;        // input pcap image
    const te_tile_t *tiles;
    const uint16_t *pkt_rel;  // record offset relative to its tile span start
    uint32_t n_tiles;
    uint32_t in_swapped, in_nsec;
    uint8_t *out;
    uint64_t out_base;        // offset of the first output record in `out`
    unsigned long long *tile_state;  // decoupled look-back granules, zeroed per launch
    unsigned int *ticket;            // zeroed per launch
    uint8_t *status;
    unsigned long long *counters;    // TE_CNT__N, zeroed per launch
    unsigned long long *err;         // [0] first error pkt, [1] its out offset, [2] look-back timeouts
    uint8_t *scratch;                // HBM slots for huge tiles
};

__device__ __forceinline__ uint32_t ld_hdr32(const uint8_t *p, bool swapped) {
    uint32_t v = ld32(p);
    return swapped ? bswap32(v) : v;
}

// ---- block-wide exclusive scan of a u32 (BLOCK threads) ----
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) {
        uint32_t s = wsum[w];
        if (w < wid) base += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// ---- decoupled look-back (single lane).  Granule = {flag:2 | value:62}
// stored/polled as one relaxed agent-scope 8-byte atomic: the value IS the
// hand-off (cdna_hip_programming.md G16 "R2"), so no fences are needed.
constexpr unsigned long long F_AGG = 1ull << 62, F_PFX = 2ull << 62, VMASK = (1ull << 62) - 1;

__device__ unsigned long long lookback(unsigned long long *state, uint32_t t, unsigned long long agg,
                                       unsigned long long *err) {
    if (t == 0) {
        __hip_atomic_store(&state[0], F_PFX | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    __hip_atomic_store(&state[t], F_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    int64_t j = (int64_t)t - 1;
    unsigned spins = 0;
    while (j >= 0) {
        unsigned long long g = __hip_atomic_load(&state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long f = g & ~VMASK;
        if (f == 0) {
            if (++spins > (1u << 26)) {  // bounded spin: report and give up
                atomicAdd(&err[2], 1ull);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += g & VMASK;
        if (f == F_PFX) break;
        --j;
    }
    __hip_atomic_store(&state[t], F_PFX | ((excl + agg) & VMASK), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// ---------------------------------------------------------------------------
// tile body.  S = slot buffer (LDS for normal tiles, HBM scratch for huge).
// ---------------------------------------------------------------------------
struct TileShared {
    uint32_t rel[TE_MAX_PKTS + 1];   // record offset in span (+ sentinel)
    uint32_t rpos[TE_MAX_PKTS];      // LDS/slot position of record start (after editing)
    uint32_t opfx[TE_MAX_PKTS + 1];  // exclusive output prefix (+ total)
    uint32_t wsum[NWAVES];
    unsigned long long cnt[TE_CNT__N];
    unsigned long long out_excl;
    uint32_t tile_id;
};

template <bool HUGE>
__device__ void tile_body(const LaunchArgs &a, const te_tile_t &tile, uint32_t t, uint8_t *S, TileShared &sh) {
    const int tid = threadIdx.x;
    const uint32_t npkt = tile.npkt;
    const uint64_t G0 = tile.span_off;  // global offset of the span
    const bool pad = a.cfg->fixlen == TE_FIXLEN_PAD;
    const bool swp = a.in_swapped != 0;

    // ---- slot layout: sizes from the record index ----
    uint32_t my_rel = 0, my_cap = 0, my_slot = 0;
    if (tid < (int)npkt) {
        my_rel = a.pkt_rel[tile.first_pkt + tid];
        uint32_t nxt = (tid + 1 < (int)npkt) ? a.pkt_rel[tile.first_pkt + tid + 1] : tile.span_len;
        my_cap = nxt - my_rel - 16;
        uint32_t data = my_cap;
        if (pad) {
            uint32_t plen = ld_hdr32(a.in + G0 + my_rel + 12, swp);
            if (plen > data) data = plen;
        }
        uint32_t g = (uint32_t)((G0 + my_rel) & 15);
        my_slot = TE_SLOT_BYTES_OF(g, data);
        sh.rel[tid] = my_rel;
    }
    if (tid == 0) sh.rel[npkt] = tile.span_len;
    uint32_t total_slot;
    uint32_t slot_base = block_exscan(my_slot, sh.wsum, total_slot);
    (void)total_slot;
    uint32_t r0 = 0;  // record start in S (before editing)
    if (tid < (int)npkt) {
        r0 = slot_base + TE_HEAD + (uint32_t)((G0 + my_rel) & 15);
        sh.rpos[tid] = r0;
    }
    __syncthreads();

    // ---- stream the span into the slots: aligned 16-byte chunks ----
    {
        const uint64_t A0 = G0 & ~15ull;
        const uint64_t Aend = G0 + tile.span_len;
        const uint32_t nchunks = (uint32_t)((Aend - A0 + 15) >> 4);
        for (uint32_t c = tid; c < nchunks; c += BLOCK) {
            const uint64_t A = A0 + ((uint64_t)c << 4);
            const uint4 v = *reinterpret_cast<const uint4 *>(a.in + A);
            // first record whose start is <= A (binary search on rel)
            int64_t rA = (int64_t)A - (int64_t)G0;
            int lo = 0, hi = (int)npkt - 1;
            while (lo < hi) {
                int mid = (lo + hi + 1) >> 1;
                if ((int64_t)sh.rel[mid] <= rA) lo = mid;
                else hi = mid - 1;
            }
            for (int p = lo; p < (int)npkt && (int64_t)sh.rel[p] < rA + 16; ++p) {
                if ((int64_t)sh.rel[p + 1] <= rA) continue;  // record ends before chunk
                const int64_t dst = (int64_t)sh.rpos[p] + (rA - (int64_t)sh.rel[p]);
                *reinterpret_cast<uint4 *>(S + dst) = v;
            }
        }
    }
    __syncthreads();

    // ---- one lane per packet ----
    uint32_t out_sz = 0;
    uint8_t st = 0;
    unsigned long long c_in = 0, c_out = 0;
    if (tid < (int)npkt) {
        uint8_t *rec = S + r0;
        uint32_t slot_end = slot_base + my_slot;
        // zero the tail (chunk stores spilled up to 15 foreign bytes into it)
        for (uint32_t i = r0 + 16 + my_cap; i < slot_end; ++i) S[i] = 0;
        uint32_t ts_sec = ld_hdr32(rec, swp), ts_frac = ld_hdr32(rec + 4, swp);
        uint32_t caplen = ld_hdr32(rec + 8, swp), len = ld_hdr32(rec + 12, swp);
        if (a.in_nsec) ts_frac /= 1000;  // libpcap opens at us precision
        c_in = 16 + (unsigned long long)caplen;
        const uint64_t pktno = a.pkt_base + tile.first_pkt + tid;  // 0-based
        int dir = TE_DIR_C2S;
        const bool explicit_dir = a.fixed_dir >= 0;
        if (explicit_dir) {
            dir = a.fixed_dir;
        } else if (a.dirbits) {  // check_cache (src/common/cache.c:321-354)
            uint64_t idx = pktno >> 2;
            uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
            uint8_t b = idx < a.dirbits_len ? a.dirbits[idx] : 0;
            dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
        }
        Pkt pk;
        pk.d = rec + 16;
        pk.caplen = caplen;
        pk.len = len;
        pk.avail = slot_end - (r0 + 16);
        pk.unsupported = false;
        int rc = RC_OK;
        bool warned = false;
        if (dir == TE_DIR_NOSEND && !explicit_dir) {  // tcprewrite.c:314-315: written unedited
            st |= TE_ST_NOSEND;
        } else {
            rc = tcpedit_packet(pk, *a.cfg, a.portlut, dir, warned);
        }
        if (pk.unsupported) st |= TE_ST_UNSUPPORTED;
        if (warned) st |= TE_ST_WARNED;
        bool write = true;
        if (rc == RC_ERROR) {
            st |= TE_ST_RC_ERROR;
            write = false;
        } else if (rc == RC_SOFT) {
            st |= TE_ST_RC_SOFT;
            if (a.cfg->skip_soft_errors) {
                st |= TE_ST_DROPPED;
                write = false;
            }
        } else if (rc == RC_WARN) {
            st |= TE_ST_RC_WARN;
        }
        if (write && pk.caplen == 0) {
            st |= TE_ST_ZEROCAP;
            write = false;
        }
        uint8_t *orec = pk.d - 16;
        st32(orec, ts_sec);
        st32(orec + 4, ts_frac);
        st32(orec + 8, pk.caplen);
        st32(orec + 12, pk.len);
        sh.rpos[tid] = (uint32_t)(orec - S);
        if (write) out_sz = 16 + pk.caplen;
        c_out = out_sz;
        a.status[tile.first_pkt + tid] = st;
    }

    // ---- tile output offsets ----
    uint32_t tile_total;
    uint32_t opos = block_exscan(out_sz, sh.wsum, tile_total);
    if (tid < (int)npkt) sh.opfx[tid] = opos;
    if (tid == 0) sh.opfx[npkt] = tile_total;

    // counters: wave reduce then LDS atomics
    {
        unsigned long long v[TE_CNT__N] = {0};
        if (tid < (int)npkt) {
            v[TE_CNT_PACKETS] = 1;
            v[TE_CNT_BYTES_IN] = c_in;
            v[TE_CNT_BYTES_OUT] = c_out;
            v[TE_CNT_WRITTEN] = out_sz ? 1 : 0;
            v[TE_CNT_EDITED] = (!(st & TE_ST_NOSEND) && (st & TE_ST_RC_MASK) <= TE_ST_RC_WARN) ? 1 : 0;
            v[TE_CNT_SOFT] = (st & TE_ST_RC_MASK) == TE_ST_RC_SOFT;
            v[TE_CNT_WARN] = (st & TE_ST_WARNED) ? 1 : 0;
            v[TE_CNT_ERROR] = (st & TE_ST_RC_MASK) == TE_ST_RC_ERROR;
            v[TE_CNT_UNSUPPORTED] = (st & TE_ST_UNSUPPORTED) ? 1 : 0;
        }
        if (tid < TE_CNT__N) sh.cnt[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < TE_CNT__N; ++k) {
            unsigned long long x = v[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((tid & 63) == 0 && x) atomicAdd(&sh.cnt[k], x);
        }
    }
    if (tid == 0) sh.out_excl = lookback(a.tile_state, t, tile_total, a.err);
    __syncthreads();
    if (tid < TE_CNT__N && sh.cnt[tid]) atomicAdd(&a.counters[tid], sh.cnt[tid]);
    const unsigned long long E = sh.out_excl;
    if (tid < (int)npkt && (st & TE_ST_RC_MASK) == TE_ST_RC_ERROR) {
        atomicMin(&a.err[0], (unsigned long long)(tile.first_pkt + tid));
        atomicMin(&a.err[1], E + opos);
    }

    // ---- stream the output records: aligned 16-byte chunks ----
    if (tile_total == 0) return;
    const uint64_t Gs = a.out_base + E;
    const uint64_t Ge = Gs + tile_total;
    const uint64_t C0 = Gs & ~15ull;
    const uint32_t nchunks = (uint32_t)((Ge - C0 + 15) >> 4);
    for (uint32_t c = tid; c < nchunks; c += BLOCK) {
        const uint64_t C = C0 + ((uint64_t)c << 4);
        const int64_t q0 = (int64_t)C - (int64_t)Gs;  // tile-relative output offset of the chunk
        const int b0 = q0 < 0 ? (int)(-q0) : 0;
        const int b1 = (C + 16 > Ge) ? (int)(Ge - C) : 16;
        // packet holding byte q0+b0
        const int64_t qf = q0 + b0;
        int lo = 0, hi = (int)npkt - 1;
        while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if ((int64_t)sh.opfx[mid] <= qf) lo = mid;
            else hi = mid - 1;
        }
        // gather the chunk's bytes from the records' slots (unrolled: registers only)
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        int p = lo;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            if (b >= b0 && b < b1) {
                const int64_t q = q0 + b;
                while ((int64_t)sh.opfx[p + 1] <= q) ++p;
                const uint32_t x = (uint32_t)S[sh.rpos[p] + (uint32_t)(q - (int64_t)sh.opfx[p])] << (8 * (b & 3));
                if (b < 4) w0 |= x;
                else if (b < 8) w1 |= x;
                else if (b < 12) w2 |= x;
                else w3 |= x;
            }
        }
        uint8_t *dst = a.out + C;
        if (b0 == 0 && b1 == 16) {
            *reinterpret_cast<uint4 *>(dst) = make_uint4(w0, w1, w2, w3);
        } else {
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                if (b >= b0 && b < b1) {
                    const uint32_t w = b < 4 ? w0 : (b < 8 ? w1 : (b < 12 ? w2 : w3));
                    dst[b] = (uint8_t)(w >> (8 * (b & 3)));
                }
            }
        }
    }
}

__global__ void __launch_bounds__(BLOCK) te_edit_tiles(LaunchArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[TE_SLOT_BYTES];
    __shared__ TileShared sh;
    for (;;) {
        if (threadIdx.x == 0) sh.tile_id = atomicAdd(a.ticket, 1u);
        __syncthreads();
        const uint32_t t = sh.tile_id;
        if (t >= a.n_tiles) return;
        const te_tile_t tile = a.tiles[t];
        if (tile.scratch_off == TE_NO_SCRATCH)
            tile_body<false>(a, tile, t, slots, sh);
        else
            tile_body<true>(a, tile, t, a.scratch + tile.scratch_off, sh);
        __syncthreads();
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI launch wrapper (called from the C host code, no torch types)
// ---------------------------------------------------------------------------
extern "C" int te_launch_edit(const te_launch_t *L, hipStream_t stream) {
    LaunchArgs a;
    a.cfg = L->cfg;
    a.portlut = L->portlut;
    a.dirbits = L->dirbits;
    a.dirbits_len = L->dirbits_len;
    a.pkt_base = L->pkt_base;
    a.fixed_dir = L->fixed_dir;
    a.in = L->in;
    a.tiles = L->tiles;
    a.pkt_rel = L->pkt_rel;
    a.n_tiles = L->n_tiles;
    a.in_swapped = L->in_swapped;
    a.in_nsec = L->in_nsec;
    a.out = L->out;
    a.out_base = L->out_base;
    a.tile_state = (unsigned long long *)L->tile_state;
    a.ticket = L->ticket;
    a.status = L->status;
    a.counters = (unsigned long long *)L->counters;
    a.err = (unsigned long long *)L->err;
    a.scratch = L->scratch;
    if (L->n_tiles == 0) return 0;
    hipError_t e = hipMemsetAsync(L->zero_region, 0, L->zero_bytes, stream);
    if (e != hipSuccess) return -1;
    // err[0], err[1] start at ~0 (atomicMin targets)
    e = hipMemsetAsync(L->err, 0xff, 2 * sizeof(uint64_t), stream);
    if (e != hipSuccess) return -1;
    int grid = L->grid > 0 ? L->grid : 1;
    if ((uint32_t)grid > L->n_tiles) grid = (int)L->n_tiles;
    hipLaunchKernelGGL(te_edit_tiles, dim3(grid), dim3(BLOCK), 0, stream, a);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : -1;
}
