// tcpedit_kernels.hip -- gfx950 kernels for the tcpedit rewrite path.
//
// One kernel, te_edit_tiles<LAYOUT>, runs the whole device pipeline of
// rewrite_packets() (src/tcprewrite.c:260-373) over a pcap image resident in
// HBM, in a single pass:
//   1. a block takes the next tile ticket (tiles = runs of consecutive records
//      whose bytes fit the block's LDS budget, built from the record index);
//   2. the tile's byte span is streamed HBM -> LDS with 16-byte loads:
//        CONTIG: the span lands as-is (one straight copy; the common case),
//        SLOT:   each record lands in its own slot with headroom/zeroed room
//                (needed only by --enet-vlan=add and --fixlen=pad), the slot
//                aligned like the record so every chunk is one 16-byte store;
//   3. one lane per packet runs tcpedit_packet() on its LDS bytes (edit_pkt.hpp);
//   4. a block scan of the output record sizes plus a decoupled look-back over
//      earlier tiles gives the tile's output offset (no second pass over HBM);
//   5. the block streams its output LDS -> HBM in 16-byte chunks, funnel-
//      shifting aligned LDS dwords; tiles whose records keep their length (the
//      common case) are one contiguous LDS -> HBM copy.
// Records too large for a tile are edited in an HBM scratch slot instead.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "edit_pkt.hpp"
#include "te_kernels.h"
#include "te_window.hpp"
#include "wave_dpp.hpp"

using namespace te;

namespace {

constexpr int BLOCK = TE_BLOCK;
constexpr int NWAVES = BLOCK / 64;
constexpr int LDS_FRONT = TE_LDS_FRONT;  // front pad so funnel reads never index below 0
constexpr int MODE_CONTIG = 0, MODE_SLOT = 1;

// explicit global / constant address spaces (device pass only): pointers
// loaded from the argument struct are otherwise generic and compile to FLAT ops
#if defined(__HIP_DEVICE_COMPILE__)
#define TE_AS_GLOBAL __attribute__((address_space(1)))
#define TE_AS_CONST __attribute__((address_space(4)))
#else
#define TE_AS_GLOBAL
#define TE_AS_CONST
#endif
typedef TE_AS_GLOBAL uint8_t g_u8;
typedef TE_AS_GLOBAL const uint8_t g_cu8;
typedef TE_AS_GLOBAL const uint4 g_cu4;
typedef TE_AS_GLOBAL uint4 g_u4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // for the nontemporal builtins
typedef TE_AS_GLOBAL u32x4 g_v4;
typedef TE_AS_GLOBAL const u32x4 g_cv4;
}  // namespace
#include "fast_lane.hpp"
namespace {

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
    unsigned long long *err;         // [0] ~first error pkt, [1] ~its out offset (0 = none), [2] look-back timeouts
    uint8_t *scratch;                // HBM slots for huge tiles
    uint64_t rec0;                   // static_off: input offset of the first record
    uint32_t static_off;             // output offsets == input offsets (size-preserving config)
    uint32_t static_grow;            // output offset = input offset + 4 x record index (VLAN add)
    uint32_t static_shrink;          // output offset = input offset - 4 x record index (VLAN pop, --efcs)
    uint32_t *grow_bad;              // set when a record breaks static_grow's placement
    // --mtu-trunc (te_launch_t.static_mtu): tile t's output at its input offset - tcut[t], the
    // predicted bytes the records before it lose; a tile whose total differs sets *grow_bad
    const long long *tcut;
    uint32_t static_mtu;
    // after te_fast_tiles: only the listed tiles are edited here, and the last
    // block folds the fast kernel's per-block counters into `counters`
    const uint32_t *tile_list;
    const uint32_t *list_cnt;        // this launch's count
    unsigned long long *counters_next;  // zeroed here for the next launch (fast lane parity)
    // --fuzz-seed: TE_FUZZ_PROBE writes status[i] = 1 for a record that reaches the fuzz
    // step and nothing else; TE_FUZZ_APPLY fuzzes record i with RNG state fuzz_state[i]
    uint32_t fuzz_mode;
    const uint32_t *fuzz_state;
    // stale static-buffer reads: a written record whose edit read bytes past
    // its physical extent is listed {record, bytes needed, output offset} for te_q8_replay
    uint4 *q8_list;
    uint32_t q8_cap;
    // per record (launch-relative index), the last C2S record's dst_modified
    // ((position << 1) | value, 0 = none yet): te_l2carry_mark + an inclusive max scan
    const unsigned long long *l2carry;
    // Q18 under --fuzz-seed: the carry's mark run (an edit pass before the edit) writes each
    // edited record's key from its own edit -- a fuzzed record's second encode writes
    // dst_modified again (tcpedit.c:89,250-258) -- over te_l2carry_mark's; null otherwise
    unsigned long long *q18_keys;
    // DLT_JUNIPER_ETHER: per record the last whole inner decode before it (te_jnpr_mark +
    // an inclusive max scan: i + 1 for record i, 0 = none in the launch, then *jctx), and
    // the states (entry i + 1: record i's); null: no carry
    const unsigned long long *jscan;
    const te_jstate_t *jstates;
    const te_jctx_t *jctx;
};

// the Juniper decoder state record j (launch-relative) is encoded with, should its frame
// be a TCPEDIT_WARN one (jnpr_ether.c:269-272)
// (and, for a fuzzed record's second decode, the state after its own first pass: the
// inclusive scan's next entry, j + 1 -- the scan has n + 1 entries)
__device__ __forceinline__ void jnpr_carry(const LaunchArgs &a, uint64_t j, Pkt &pk) {
    if (!a.jscan) return;
    const unsigned long long i = a.jscan[j], i2 = a.jscan[j + 1];
    const uint32_t v = a.jctx->valid;
    if (i) {
        pk.jc = &a.jstates[i];
    } else {
        if (v == TE_JC_VALID) pk.jc = &a.jctx->st;
        else if (v == TE_JC_NONE) pk.jnone = true;
    }
    if (i2) {
        pk.jc2 = &a.jstates[i2];
    } else {
        if (v == TE_JC_VALID) pk.jc2 = &a.jctx->st;
        else if (v == TE_JC_NONE) pk.jnone2 = true;
    }
}

__device__ __forceinline__ uint32_t ld_hdr32(const uint8_t *p, bool swapped) {
    uint32_t v = ld32(p);
    return swapped ? bswap32(v) : v;
}

// unsigned min (HIP's min() of mixed int/unsigned arguments resolves to the double overload)
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// ---- block-wide exclusive scan of a u32 (NT threads) ----
template <int NT = BLOCK>
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
    for (int w = 0; w < NT / 64; ++w) {
        uint32_t s = wsum[w];
        if (w < wid) base += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// ---- decoupled look-back, one wave.  Granule = {flag:2 | value:62} stored/
// polled as one relaxed agent-scope 8-byte atomic: the value IS the hand-off
// (cdna_hip_programming.md G16 "R2"), so no fences are needed.  Each round
// polls the 64 nearest unresolved predecessors at once (lane k = tile j-k):
// one cross-XCD round trip per 64 tiles of depth instead of one per tile.
// Called by all 64 lanes of wave 0; returns the exclusive prefix on every lane.
constexpr unsigned long long F_AGG = 1ull << 62, F_PFX = 2ull << 62, VMASK = (1ull << 62) - 1;

__device__ __forceinline__ unsigned long long lookback(unsigned long long *state, uint32_t t, unsigned long long agg,
                                                       unsigned long long *err) {
    const int lane = threadIdx.x & 63;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(&state[0], F_PFX | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&state[t], F_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    int64_t j = (int64_t)t - 1;  // nearest unresolved predecessor
    unsigned spins = 0;
    while (j >= 0) {
        const int64_t idx = j - lane;
        unsigned long long g = F_PFX;  // before tile 0: prefix 0
        if (idx >= 0) g = __hip_atomic_load(&state[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long f = g & ~VMASK;
        const unsigned long long pm = __ballot(f == F_PFX), zm = __ballot(f == 0);
        const int first_p = pm ? __builtin_ctzll(pm) : 64;
        const int first_z = zm ? __builtin_ctzll(zm) : 64;
        const int take = first_z < first_p ? first_z : (first_p < 64 ? first_p + 1 : 64);
        unsigned long long v = lane < take ? (g & VMASK) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (first_p < first_z) break;  // reached an inclusive prefix
        j -= take;
        if (first_z < 64) {  // a predecessor has not published yet
            if (++spins > (1u << 24)) {  // bounded spin: report and give up
                if (lane == 0) atomicAdd(&err[2], 1ull);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0)
        __hip_atomic_store(&state[t], F_PFX | ((excl + agg) & VMASK), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

constexpr int JPIECE = 64;                                       // bytes of a deferred-sum piece
constexpr int JMAP = (TE_SLOT_BYTES + 64) / JPIECE + TE_MAX_PKTS;  // pieces of a tile, at most
struct TileShared {
    uint32_t rel[TE_MAX_PKTS + 1];   // record offset in span (+ sentinel); after the span load:
                                     // each record's deferred L4 sum (the pieces' folded sums)
    uint32_t rpos[TE_MAX_PKTS];      // slot position of the output record start
    uint32_t opfx[TE_MAX_PKTS + 1];  // exclusive output prefix (+ total); before the placement:
                                     // each record's deferred L4 sum start (slot offset)
    uint32_t wsum[NWAVES];
    unsigned long long cnt[TE_CNT__N];
    unsigned long long out_excl;
    uint32_t tile_id;
    uint32_t ident;                  // every record kept its input size (contiguous output)
};

// the LDS tile path's deferred L4 sums: per record (bytes << 16 | first piece), piece -> record;
// then (the sums done) the store's output chunk -> the record holding its first byte
constexpr int CMAP = (TE_SLOT_BYTES + LDS_FRONT + 64) / 16 + 2;
struct JobShared {
    union {
        struct {
            uint32_t jlp[TE_MAX_PKTS];
            uint8_t jmap[JMAP];
        };
        uint8_t cmap[CMAP];
    };
};

// 16 bytes of the slot buffer starting at byte `base` (any alignment): five
// aligned dword reads and four byte-funnel shifts.
template <typename P>
__device__ __forceinline__ uint4 read16(P S, uint32_t base) {
    const uint32_t a = base & ~3u, sh = base & 3u;
    const uint32_t *w = (const uint32_t *)(S + a);
    uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    if (sh == 0) return make_uint4(w0, w1, w2, w3);
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

__device__ __forceinline__ uint32_t sel_bytes(uint32_t x, uint32_t y, int b0, int b1, int k) {
    // bytes [b0,b1) of dword k (bytes 4k..4k+3) from y, the rest from x
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int b = 4 * k + i;
        if (b >= b0 && b < b1) m |= 0xffu << (8 * i);
    }
    return (x & ~m) | (y & m);
}

#ifndef TE_GK_LOAD_K
#define TE_GK_LOAD_K 5
#endif
// TE_GK_STAMPS builds (diagnostics only): s_memtime per tile phase, wave 0's view (so a
// phase includes the barrier wait behind it), summed per block, printed by a few blocks
#if TE_GK_STAMPS
__shared__ unsigned long long gk_ph[6], gk_last;
#define GK_STAMP(i)                                                        \
    if (threadIdx.x == 0) {                                                \
        __builtin_amdgcn_sched_barrier(0);                                 \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
        __builtin_amdgcn_sched_barrier(0);                                 \
        gk_ph[i] += now_ - gk_last;                                        \
        gk_last = now_;                                                    \
    }
#else
#define GK_STAMP(i)
#endif

// ---------------------------------------------------------------------------
// tile body.  S = slot buffer (LDS, or HBM scratch for a huge record).
// ---------------------------------------------------------------------------
template <int MODE, bool FZ, typename P, bool AD = false>
__device__ __forceinline__ void tile_body(const LaunchArgs &a, const te_tile_t &tile, uint32_t t, P S,
                                          TileShared &sh, const te_dev_cfg_t &cfg, JobShared *js) {
    const int tid = threadIdx.x;
    const uint32_t npkt = tile.npkt;
    const uint64_t G0 = tile.span_off;  // HBM offset of the span
    const uint64_t A0 = G0 & ~15ull;    // first aligned chunk
    const bool swp = a.in_swapped != 0;
    g_cu8 *gin = (g_cu8 *)a.in;

    // ---- record positions ----
    uint32_t my_rel = 0, my_cap = 0, my_slot = 0, r0 = 0, slot_end = 0;
    if (tid < (int)npkt) {
        my_rel = a.pkt_rel[tile.first_pkt + tid];
        uint32_t nxt = (tid + 1 < (int)npkt) ? a.pkt_rel[tile.first_pkt + tid + 1] : tile.span_len;
        my_cap = nxt - my_rel - 16;
        sh.rel[tid] = my_rel;
    }
    if (tid == 0) sh.rel[npkt] = tile.span_len;
    if constexpr (MODE == MODE_SLOT) {
        if (tid < (int)npkt) {
            uint32_t data = my_cap;
            if (cfg.fixlen == TE_FIXLEN_PAD) {
                const g_cu8 *lp = gin + G0 + my_rel + 12;
                uint32_t plen = (uint32_t)lp[0] | ((uint32_t)lp[1] << 8) | ((uint32_t)lp[2] << 16) |
                                ((uint32_t)lp[3] << 24);
                if (swp) plen = bswap32(plen);
                if (plen > data) data = plen;
            }
            my_slot = TE_SLOT_BYTES_OF_H(cfg.slot_head, (uint32_t)((G0 + my_rel) & 15), data);
        }
        uint32_t total_slot;
        uint32_t slot_base = LDS_FRONT + block_exscan(my_slot, sh.wsum, total_slot);
        if (tid < (int)npkt) {
            r0 = slot_base + cfg.slot_head + (uint32_t)((G0 + my_rel) & 15);
            slot_end = slot_base + my_slot;
            sh.rpos[tid] = r0;
        }
    } else {
        if (tid < (int)npkt) {
            r0 = LDS_FRONT + (uint32_t)(G0 - A0) + my_rel;
            slot_end = r0 + 16 + my_cap;
            sh.rpos[tid] = r0;
        }
    }
    __syncthreads();

    GK_STAMP(0);  // positions
    // ---- stream the span into LDS: aligned 16-byte chunks ----
    {
        const uint64_t Aend = G0 + tile.span_len;
        const uint32_t nchunks = (uint32_t)((Aend - A0 + 15) >> 4);
        if constexpr (MODE == MODE_CONTIG) {
            // every chunk a lane owns is in flight before the first LDS store: one HBM
            // round trip per tile instead of one per chunk
            constexpr int K = TE_GK_LOAD_K;  // 16-byte chunks per lane per batch
            for (uint32_t c0 = tid; c0 < nchunks; c0 += K * BLOCK) {
                uint4 v[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {  // unconditional (clamped) loads keep v[] in VGPRs
                    const uint32_t c = umin32(c0 + k * BLOCK, nchunks - 1u);
                    v[k] = *(g_cu4 *)(gin + A0 + ((uint64_t)c << 4));
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const uint32_t c = c0 + k * BLOCK;
                    if (c < nchunks) *(uint4 *)(S + LDS_FRONT + (c << 4)) = v[k];
                }
            }
        }
        for (uint32_t c = tid; MODE != MODE_CONTIG && c < nchunks; c += BLOCK) {
            const uint64_t A = A0 + ((uint64_t)c << 4);
            const uint4 v = *(g_cu4 *)(gin + A);
            {
                int64_t rA = (int64_t)A - (int64_t)G0;
                int lo = 0, hi = (int)npkt - 1;
                while (lo < hi) {
                    int mid = (lo + hi + 1) >> 1;
                    if ((int64_t)sh.rel[mid] <= rA) lo = mid;
                    else hi = mid - 1;
                }
                for (int p = lo; p < (int)npkt && (int64_t)sh.rel[p] < rA + 16; ++p) {
                    if ((int64_t)sh.rel[p + 1] <= rA) continue;
                    const int64_t dst = (int64_t)sh.rpos[p] + (rA - (int64_t)sh.rel[p]);
                    *(uint4 *)(S + dst) = v;
                }
            }
        }
    }
    __syncthreads();
    GK_STAMP(1);  // span load

    // ---- one lane per packet ----
    uint32_t out_sz = 0, need = 0;
    uint8_t st = 0;
    unsigned long long c_in = 0;
    // deferred L4 sums: the LDS tile path only (a huge record's HBM slot sums in its lane)
    constexpr bool kDefer = __is_same(P, uint8_t *);
    bool job = false;
    uint8_t *job_l4 = nullptr, *job_field = nullptr;
    uint32_t job_base = 0, njob = 0;
    if (tid < (int)npkt) {
        uint8_t *rec = (uint8_t *)(S + r0);
        if constexpr (MODE == MODE_SLOT)  // zero the room after the data (chunk stores spilled into it)
            for (uint32_t i = r0 + 16 + my_cap; i < slot_end; ++i) S[i] = 0;
        uint32_t ts_sec = ld_hdr32(rec, swp), ts_frac = ld_hdr32(rec + 4, swp);
        const uint32_t fcap = ld_hdr32(rec + 8, swp), len = ld_hdr32(rec + 12, swp);
        if (a.in_nsec) ts_frac /= 1000;  // libpcap opens at us precision
        c_in = 16 + (unsigned long long)fcap;
        // safe_pcap_next (src/common/utils.c:159-162): len < caplen -> caplen = len before
        // tcprewrite.c:301's copy, so the bytes past it are not the record's (a read there
        // is a stale static-buffer read, Q8)
        const uint32_t caplen = len < fcap ? len : fcap;
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
        pk.phys = my_cap < caplen ? my_cap : caplen;
        pk.avail = slot_end - (r0 + 16);
        pk.unsupported = false;
        pk.need = 0;
        pk.ext = caplen;
        pk.strict = false;
        // the slot's headroom and the record's 16-byte alignment gap (slot layouts); a
        // contiguous span has no byte before a record that is the record's own
        pk.room = MODE == MODE_SLOT ? r0 - (slot_end - my_slot) : 0u;
        pk.l2carry = a.l2carry ? (uint8_t)(a.l2carry[tile.first_pkt + tid] & 1u) : 0;
        if (FZ && AD && a.l2carry && (a.l2carry[tile.first_pkt + tid] >> 63))
            stale(pk, (int)NEED_NEVER);  // a poisoned carry (q18_keys): fails loudly
        if constexpr (AD) jnpr_carry(a, tile.first_pkt + tid, pk);
        pk.defer = kDefer;
        int rc = RC_OK;
        bool warned = false;
        if (dir == TE_DIR_NOSEND && !explicit_dir) {  // tcprewrite.c:314-315: written unedited
            st |= TE_ST_NOSEND;
        } else {
            const uint32_t fzs = a.fuzz_mode == TE_FUZZ_APPLY ? a.fuzz_state[tile.first_pkt + tid] : 0u;
            rc = tcpedit_packet<FZ, AD>(pk, cfg, (const TE_AS_GLOBAL uint16_t *)a.portlut, dir, warned,
                                        a.fuzz_mode, fzs);
            if (FZ && AD && a.q18_keys) {  // (the carry's decoders are the ANYDEC instance's)
                // the record's last dst_modified write; a stale read before a write in its
                // second pass poisons the carry from here on (bit 63: the edit run fails
                // those records loudly rather than guess what the bytes would have decided)
                const uint32_t j = tile.first_pkt + tid;
                unsigned long long k = (pk.q18ev & 2u) ? ((unsigned long long)(j + 1) << 1 | (pk.q18ev & 1u)) : 0ull;
                if (pk.unsupported && (pk.q18ev & 6u) == 6u) k |= 1ull << 63;
                a.q18_keys[j + 1] = k;
            }
        }
        if (FZ && a.fuzz_mode == TE_FUZZ_PROBE) st = rc == RC_REACHED ? 1 : 0;
        if (warned) st |= TE_ST_WARNED;
        bool write = true;
        if (rc == RC_ERROR) {
            st |= TE_ST_RC_ERROR;
            write = false;
        } else if (rc == RC_SOFT) {
            st |= TE_ST_RC_SOFT;
            if (cfg.skip_soft_errors) {
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
        // a stale read only matters when the record is written (its bytes are the output)
        if (pk.unsupported && write && !(FZ && a.fuzz_mode == TE_FUZZ_PROBE)) {
            st |= TE_ST_UNSUPPORTED;
            need = pk.need;
        }
        uint8_t *orec = pk.d - 16;
        if (swp || a.in_nsec || pk.d != rec + 16) {
            st32(orec, ts_sec);
            st32(orec + 4, ts_frac);
        }
        if (swp || pk.caplen != fcap || pk.len != len || pk.d != rec + 16) {
            st32(orec + 8, pk.caplen);
            st32(orec + 12, pk.len);
        }
        sh.rpos[tid] = (uint32_t)(orec - (uint8_t *)S);
        if (write) out_sz = 16 + pk.caplen;
        ((g_u8 *)a.status)[tile.first_pkt + tid] = st;
        if constexpr (kDefer) {
            job = pk.job_field != nullptr;
            job_l4 = pk.job_l4;
            job_field = pk.job_field;
            job_base = pk.job_base;
            njob = job ? (uint32_t)pk.job_len : 0u;
        }
    }
    GK_STAMP(2);  // edit (wave 0's lanes)
    if (FZ && a.fuzz_mode == TE_FUZZ_PROBE) return;  // the reach pass writes nothing else

    // ---- the deferred L4 payload sums (do_checksum, checksum.c:34-170): one packet a lane
    // left a 1514-byte sum to one lane while its neighbours' 64-byte packets were done, so
    // every record's payload is cut into 64-byte pieces and the block's 256 threads sum the
    // pieces (aligned LDS quads, absolute weights), adding each into its record's slot;
    // then each lane writes its checksum field as csum_bytes + CHECKSUM_CARRY would ----
    if constexpr (kDefer) {
        uint32_t npiece = (njob + JPIECE - 1) / JPIECE, tot_pieces;
        const uint32_t pb = block_exscan(npiece, sh.wsum, tot_pieces);
        if (tot_pieces) {  // (block-uniform)
            // (tot_pieces <= sum of ceil(len / 64) <= slot bytes / 64 + records = JMAP)
            if (tid < (int)npkt) {
                sh.opfx[tid] = (uint32_t)(job_l4 - (uint8_t *)S);
                js->jlp[tid] = njob << 16 | pb;
                sh.rel[tid] = 0;
                for (uint32_t q = 0; q < npiece; ++q) js->jmap[pb + q] = (uint8_t)tid;
            }
            __syncthreads();
            for (uint32_t p = tid; p < tot_pieces; p += BLOCK) {
                const uint32_t j = js->jmap[p], lp = js->jlp[j];
                const uint32_t off = (p - (lp & 0xffffu)) * JPIECE, n = umin32(JPIECE, (lp >> 16) - off);
                const uint8_t *pp = (const uint8_t *)S + sh.opfx[j] + off;
                atomicAdd(&sh.rel[j], fold16(sum_abs(pp, (int)n)));
            }
            __syncthreads();
            if (job) st16(job_field, csum_carry((unsigned long long)job_base + csum_of_job(job_l4, sh.rel[tid])));
        }
    }

    // ---- tile output offsets ----
    // static_off: sizes are preserved, so output offsets are the input offsets
    // (no scan, no look-back); otherwise block scan + decoupled look-back.
    const bool stat = a.static_off != 0, shrink = a.static_shrink != 0, grow = a.static_grow != 0 || shrink;
    uint32_t tile_total, opos;
    bool keep = true;
    if (MODE == MODE_CONTIG && stat) {
        opos = my_rel;
        tile_total = tile.span_len;
        if (tid < TE_CNT__N) sh.cnt[tid] = 0;
        __syncthreads();
    } else if (grow) {
        // every record before this one grew (shrank) by 4 bytes (or the output ends at an
        // earlier hard error): static placement, checked record by record
        opos = shrink ? my_rel - 4u * (uint32_t)tid : my_rel + 4u * (uint32_t)tid;
        tile_total = shrink ? tile.span_len - 4u * npkt : tile.span_len + 4u * npkt;
        if (tid < (int)npkt) {
            sh.opfx[tid] = opos;
            if ((st & TE_ST_RC_MASK) != TE_ST_RC_ERROR && out_sz != (shrink ? 16 + my_cap - 4 : 16 + my_cap + 4))
                atomicOr(a.grow_bad, 1u);
        }
        if (tid == 0) {
            sh.opfx[npkt] = tile_total;
            sh.ident = 0;
        }
        if (tid < TE_CNT__N) sh.cnt[tid] = 0;
        __syncthreads();
    } else {
        keep = tid >= (int)npkt || (out_sz == 16 + my_cap && sh.rpos[tid] == r0);
        opos = block_exscan(out_sz, sh.wsum, tile_total);
        if (tid < (int)npkt) sh.opfx[tid] = opos;
        if (tid == 0) {
            sh.opfx[npkt] = tile_total;
            sh.ident = 1;
        }
        if (tid < TE_CNT__N) sh.cnt[tid] = 0;
        __syncthreads();
        if (!keep) sh.ident = 0;  // benign race: every writer stores 0
    }

    // counters: wave reduce then LDS atomics
    {
        unsigned long long v[TE_CNT__N];
        const bool on = tid < (int)npkt;
        v[TE_CNT_PACKETS] = on;
        v[TE_CNT_BYTES_IN] = c_in;
        v[TE_CNT_BYTES_OUT] = out_sz;
        v[TE_CNT_WRITTEN] = out_sz ? 1 : 0;
        v[TE_CNT_EDITED] = on && !(st & TE_ST_NOSEND) && (st & TE_ST_RC_MASK) <= TE_ST_RC_WARN;
        v[TE_CNT_SOFT] = on && (st & TE_ST_RC_MASK) == TE_ST_RC_SOFT;
        v[TE_CNT_WARN] = (st & TE_ST_WARNED) ? 1 : 0;
        v[TE_CNT_ERROR] = on && (st & TE_ST_RC_MASK) == TE_ST_RC_ERROR;
        v[TE_CNT_UNSUPPORTED] = 0;  // counted per record below (the q8 list index)
        v[TE_CNT_Q8_FAILED] = 0;
#pragma unroll
        for (int k = 0; k < TE_CNT__N; ++k) {
            unsigned long long x = v[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((tid & 63) == 0 && x) atomicAdd(&sh.cnt[k], x);
        }
    }
    if (stat || grow) {
        if (tid == 0)
            sh.out_excl = tile.span_off - a.rec0 +
                          (shrink ? -4ull * tile.first_pkt : (grow ? 4ull * tile.first_pkt : 0ull));
    } else if (a.static_mtu) {  // the predicted placement, checked by the tile's total
        if (tid == 0) {
            const long long c0 = a.tcut[t], c1 = a.tcut[t + 1];
            sh.out_excl = (unsigned long long)((long long)(tile.span_off - a.rec0) - c0);
            if ((long long)tile_total != (long long)tile.span_len - (c1 - c0)) atomicOr(a.grow_bad, 1u);
        }
    } else if (tid < 64) {
        const unsigned long long e = lookback(a.tile_state, t, tile_total, a.err);
        if (tid == 0) sh.out_excl = e;
    }
    __syncthreads();
    if (tid < TE_CNT__N && sh.cnt[tid]) atomicAdd(&a.counters[tid], sh.cnt[tid]);
    const unsigned long long E = sh.out_excl;
    if (tid < (int)npkt && (st & TE_ST_RC_MASK) == TE_ST_RC_ERROR) {
        // zero-initialised words hold ~value: atomicMax(~x) == ~min(x)
        atomicMax(&a.err[0], ~(unsigned long long)(tile.first_pkt + tid));
        atomicMax(&a.err[1], ~(a.out_base + E + opos));
    }
    if (tid < (int)npkt && (st & TE_ST_UNSUPPORTED)) {  // rare: one global atomic per record
        const unsigned long long k = atomicAdd(&a.counters[TE_CNT_UNSUPPORTED], 1ull);
        const unsigned long long o = a.out_base + E + opos;
        if (a.q8_list && k < a.q8_cap)
            a.q8_list[k] = make_uint4(tile.first_pkt + tid, need, (uint32_t)o, (uint32_t)(o >> 32));
    }

    GK_STAMP(3);  // placement, counters, look-back
    // ---- stream the output records: aligned 16-byte chunks ----
    if (tile_total == 0) return;
    const uint64_t Gs = a.out_base + E;
    const uint64_t Ge = Gs + tile_total;
    const uint64_t C0 = Gs & ~15ull;
    const uint32_t nchunks = (uint32_t)((Ge - C0 + 15) >> 4);
    const bool ident = MODE == MODE_CONTIG && (stat || sh.ident != 0);
    const uint32_t src0 = sh.rpos[0];  // ident: output byte q is slot byte src0 + q
    g_u8 *gout = (g_u8 *)a.out;
    if (kDefer && !ident) {
        // the chunk map: every record marks the output chunks whose first byte it holds
        // (chunk c's first byte is tile byte max(16 c - g, 0)), so a chunk finds its first
        // record in one LDS read instead of a binary search over the tile's records
        const uint32_t g = (uint32_t)(Gs - C0);
        if (tid < (int)npkt) {
            const uint32_t s0 = sh.opfx[tid], s1 = sh.opfx[tid + 1];
            if (s1 > s0) {
                const uint32_t c_lo = s0 == 0 ? 0u : (s0 + g + 15) >> 4, c_hi = (s1 + g + 15) >> 4;
                for (uint32_t c = c_lo; c < c_hi && c < (uint32_t)CMAP; ++c) js->cmap[c] = (uint8_t)tid;
            }
        }
        __syncthreads();
    }
    for (uint32_t c = tid; c < nchunks; c += BLOCK) {
        const uint64_t C = C0 + ((uint64_t)c << 4);
        const int64_t q0 = (int64_t)C - (int64_t)Gs;  // tile-relative output offset of the chunk
        const int b0 = q0 < 0 ? (int)(-q0) : 0;
        const int b1 = (C + 16 > Ge) ? (int)(Ge - C) : 16;
        uint4 v;
        if (ident) {
            v = read16(S, (uint32_t)((int64_t)src0 + q0));
        } else {
            // records overlapping the chunk: the first from the chunk map (the HBM slot path:
            // a binary search), then walk
            const int64_t qf = q0 + b0;
            int lo = 0, hi = (int)npkt - 1;
            if (kDefer) {
                lo = js->cmap[c];
            } else {
                while (lo < hi) {
                    int mid = (lo + hi + 1) >> 1;
                    if ((int64_t)sh.opfx[mid] <= qf) lo = mid;
                    else hi = mid - 1;
                }
            }
            v = make_uint4(0, 0, 0, 0);
            const int64_t f0 = sh.opfx[lo], f1 = sh.opfx[lo + 1];
            if (f0 <= q0 && f1 >= q0 + 16) {
                // the whole chunk inside one record (most chunks): one read, no byte selects
                v = read16(S, (uint32_t)((int64_t)sh.rpos[lo] + (q0 - f0)));
            } else {
                for (int p = lo; p < (int)npkt && (int64_t)sh.opfx[p] < q0 + b1; ++p) {
                    const int64_t s0 = sh.opfx[p], s1 = sh.opfx[p + 1];
                    if (s1 <= q0 + b0) continue;
                    int pb0 = (int)((s0 - q0) > b0 ? (s0 - q0) : b0);
                    int pb1 = (int)((s1 - q0) < b1 ? (s1 - q0) : b1);
                    if (pb0 >= pb1) continue;
                    const uint4 w = read16(S, (uint32_t)((int64_t)sh.rpos[p] + (q0 - s0)));
                    v.x = sel_bytes(v.x, w.x, pb0, pb1, 0);
                    v.y = sel_bytes(v.y, w.y, pb0, pb1, 1);
                    v.z = sel_bytes(v.z, w.z, pb0, pb1, 2);
                    v.w = sel_bytes(v.w, w.w, pb0, pb1, 3);
                }
            }
        }
        g_u8 *dst = gout + C;
        if (b0 == 0 && b1 == 16) {
            *(g_u4 *)dst = v;
        } else {
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                if (b >= b0 && b < b1) {
                    const uint32_t w = b < 4 ? v.x : (b < 8 ? v.y : (b < 12 ? v.z : v.w));
                    dst[b] = (uint8_t)(w >> (8 * (b & 3)));
                }
            }
        }
    }
    GK_STAMP(4);  // output store
}

// records larger than a tile: same body over an HBM scratch slot, kept out of
// line.  The arguments are read through the kernel's kernarg segment, whose
// address the kernel passes in: the kernarg-pointer builtin is only defined in
// a kernel entry (a callee gets null), and taking &a in the kernel would copy
// the arguments to scratch for every tile.
template <bool FZ, bool AD>
__device__ __attribute__((noinline)) void huge_tile(const TE_AS_CONST LaunchArgs *ka, uint32_t t,
                                                    const te_dev_cfg_t &cfg) {
    const LaunchArgs &a = *(const LaunchArgs *)ka;
    __shared__ TileShared hsh;
    const te_tile_t tile = a.tiles[t];
    tile_body<MODE_SLOT, FZ, g_u8 *, AD>(a, tile, t, (g_u8 *)(a.scratch + tile.scratch_off), hsh, cfg, nullptr);
}

#ifndef TE_MIN_WAVES
#define TE_MIN_WAVES 3
#endif
// AD: the instance that also carries the non-Ethernet decoders and encoders (tcpedit_packet)
template <int MODE, bool FZ = false, bool AD = false>
__global__ void __launch_bounds__(BLOCK, TE_MIN_WAVES) te_edit_tiles(LaunchArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[TE_SLOT_BYTES + LDS_FRONT + 64];
    __shared__ TileShared sh;
    __shared__ JobShared js;
    __shared__ __attribute__((aligned(16))) te_dev_cfg_t cfg;  // per-run tables, read uniformly by every lane
    const bool listed = a.tile_list != nullptr;
    if (a.counters_next && blockIdx.x == 0 && threadIdx.x < TE_CNT__N) a.counters_next[threadIdx.x] = 0;
    const uint32_t n_work = listed ? *(const volatile uint32_t *)a.list_cnt : a.n_tiles;
    if (n_work == 0) return;  // after the fast lane, usually nothing is left
    {
        static_assert(sizeof(te_dev_cfg_t) % 4 == 0, "cfg copy");
        const uint32_t *src = (const uint32_t *)a.cfg;
        uint32_t *dst = (uint32_t *)&cfg;
        for (int i = threadIdx.x; i < (int)(sizeof(te_dev_cfg_t) / 4); i += BLOCK) dst[i] = src[i];
    }
#if TE_GK_STAMPS
    uint32_t gk_nt = 0;
    if (threadIdx.x == 0) {
        for (int i = 0; i < 6; ++i) gk_ph[i] = 0;
        gk_last = __builtin_amdgcn_s_memtime();
    }
#endif
    for (;;) {
        if (threadIdx.x == 0) sh.tile_id = atomicAdd(a.ticket, 1u);
        __syncthreads();
        uint32_t t = sh.tile_id;
        __syncthreads();
        GK_STAMP(5);  // ticket + the previous tile's tail
        if (t >= n_work) break;
#if TE_GK_STAMPS
        ++gk_nt;
#endif
        if (listed) t = a.tile_list[t];
        const te_tile_t tile = a.tiles[t];
        if (tile.scratch_off == TE_NO_SCRATCH)
            tile_body<MODE, FZ, uint8_t *, AD>(a, tile, t, slots, sh, cfg, &js);
        else
            huge_tile<FZ, AD>((const TE_AS_CONST LaunchArgs *)__builtin_amdgcn_kernarg_segment_ptr(), t, cfg);
        __syncthreads();
    }
#if TE_GK_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 4)
        printf("GK block %u tiles %u pos %llu load %llu edit %llu place %llu store %llu ticket %llu\n", blockIdx.x,
               gk_nt, gk_ph[0], gk_ph[1], gk_ph[2], gk_ph[3], gk_ph[4], gk_ph[5]);
#endif
}

// ===========================================================================
// te_packet_server: tcpedit_packet (tcpedit.c:46-366) for a caller that edits one record
// a call.  A launch, a copy each way and a stream sync cost ~100 us a call; this block
// stays resident instead and serves requests through host-mapped memory (te_srv_ctl_t):
// the record is read over PCIe straight from the caller-side staging buffer, edited in
// LDS by the generic lane's tile body (one tile of one record, slot layout, every
// decoder), and written back over PCIe.  Acquire/release at system scope order the
// request and response words with the bytes.  The loop ends on `stop` or after
// idle_ticks without a request, so the grid always drains.
// ===========================================================================
static_assert(offsetof(te_srv_ctl_t, seq) == 0 && offsetof(te_srv_ctl_t, stop) == 4 && offsetof(te_srv_ctl_t, dir) == 8 &&
                  offsetof(te_srv_ctl_t, caplen) == 12,
              "the server polls {seq, stop, dir, caplen} as one 16-byte word (the control block is page-aligned)");
__global__ void __launch_bounds__(BLOCK) te_packet_server(te_srv_launch_t s) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[TE_SLOT_BYTES + LDS_FRONT + 64];
    __shared__ TileShared sh;
    __shared__ JobShared js;
    __shared__ __attribute__((aligned(16))) te_dev_cfg_t cfg;
    __shared__ uint32_t req, quit;
    {
        const uint32_t *src = (const uint32_t *)s.cfg;
        uint32_t *dst = (uint32_t *)&cfg;
        for (int i = threadIdx.x; i < (int)(sizeof(te_dev_cfg_t) / 4); i += BLOCK) dst[i] = src[i];
    }
    te_srv_ctl_t *ctl = s.ctl;
    unsigned long long *cnt = (unsigned long long *)(s.scratch + 64);
    LaunchArgs a = {};
    a.cfg = s.cfg;
    a.portlut = s.portlut;
    a.in = s.in;
    a.out = s.out;
    a.out_base = 24;
    a.status = s.scratch;
    a.counters = cnt;
    a.err = cnt + TE_CNT__N;
    a.tile_state = cnt + TE_CNT__N + 4;
    a.pkt_rel = (const uint16_t *)(s.scratch + 16);  // one zero word
    a.n_tiles = 1;
    a.fuzz_mode = TE_FUZZ_OFF;
    a.pkt_base = 0;  // (a fixed direction: no tcpprep cache lookup by packet number)
    __shared__ uint32_t rq_dir, rq_caplen;
    uint32_t last = s.start_seq;
    for (;;) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t q = 0;
            u32x4 w;
            for (;;) {
                // {seq, stop, dir, caplen} in one read over PCIe: the request rides with its seq
                w = *(const volatile u32x4 *)ctl;
                if (w.x != last) break;
                if (w.y || __builtin_amdgcn_s_memrealtime() - t0 > s.idle_ticks) {
                    q = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            req = w.x;
            quit = q;
            rq_dir = w.z;
            rq_caplen = w.w;
        }
        __syncthreads();
        if (quit) break;
        // the host's stores before its release of seq (the record) are visible from here on
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t seq = req;
        const uint32_t caplen = rq_caplen;
        a.fixed_dir = (int32_t)rq_dir;
        te_tile_t tile;
        tile.span_off = 24;
        tile.scratch_off = TE_NO_SCRATCH;
        tile.first_pkt = 0;
        tile.npkt = 1;
        tile.span_len = 16 + caplen;
        tile.flags = 0;
        tile_body<MODE_SLOT, false, uint8_t *, true>(a, tile, 0, slots, sh, cfg, &js);
        __syncthreads();  // (the block's counters are in sh.cnt)
        if (threadIdx.x == 0) {
            ctl->status = *(volatile uint8_t *)s.scratch;  // (this lane's own store: the record's lane)
            ctl->bytes_out = sh.cnt[TE_CNT_BYTES_OUT];
            ctl->packets = sh.cnt[TE_CNT_PACKETS];
            ctl->edited = sh.cnt[TE_CNT_EDITED];
        }
        // every lane's output stores and the response words are complete and visible to the
        // host (one PCIe round trip for all of them) before done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(&ctl->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = seq;
        __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(&ctl->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ===========================================================================
// te_fast_tiles: the register-resident fast lane (fast_lane.hpp) over tiles of
// a size-preserving run (static offsets).  Lean on purpose -- few VGPRs and a
// small LDS image, so many blocks per CU hide HBM latency.  A tile holding any
// packet the fast lane does not carry (or a huge record) is not written here:
// its id goes to tile_list and the generic kernel, launched next, redoes the
// whole tile (its results for the fast-lane packets are the same bytes).
// ===========================================================================
#ifndef TE_FK_PREFETCH
#define TE_FK_PREFETCH 1  // load tile k+1 into registers while tile k is edited
#endif
#ifndef TE_FK_MIN_BLOCKS
#define TE_FK_MIN_BLOCKS 3  // waves per SIMD (the second launch-bounds argument on this toolchain)
#endif
constexpr int FKB = TE_FK_BLOCK;                              // threads per fast-lane block
constexpr int FK_LDS = TE_FK_TILE_BYTES + LDS_FRONT + 128;  // + window overrun past the span
constexpr int FK_NCH = (TE_FK_TILE_BYTES + LDS_FRONT + 15) / 16 + 2;
constexpr int FK_Q = (FK_NCH + FKB - 1) / FKB;

// TE_FK_STAMPS builds (diagnostics only): s_memtime per phase, summed per block,
// printed by a few blocks at exit
#if TE_FK_STAMPS
#define FK_STAMP(i)                                     \
    {                                                   \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        ph[i] += now_ - last_;                          \
        last_ = now_;                                   \
    }
#else
#define FK_STAMP(i)
#endif

struct FastArgs {
    const te_dev_cfg_t *cfg;
    const uint16_t *portlut;
    const uint8_t *dirbits;
    uint64_t dirbits_len;
    uint64_t pkt_base;
    const uint8_t *in;
    const te_tile_t *tiles;
    const uint16_t *pkt_rel;
    uint8_t *out;
    uint8_t *status;
    uint32_t *tile_list;
    uint32_t *list_cnt;  // this launch's count; list_cnt_next is zeroed for the next launch
    uint32_t *list_cnt_next;
    unsigned long long *counters;  // this launch's counter set (zeroed by the previous launch)
    unsigned long long *slots;     // te_wave_tiles: per-block totals (TE_WK_SLOT_WORDS a block), summed by the host
    unsigned long long *counters_next;  // te_wave_tiles: the other parity's counter set, zeroed for the next launch
    unsigned long long *ws_zero;
    uint64_t out_base, rec0;
    uint32_t n_tiles;
    int32_t fixed_dir;
    uint32_t in_swapped, in_nsec, v6_ok;
    uint32_t seed_sw, seed_on, skip_bcast;  // te_wave_tiles' phase-A knobs (fl::Knobs), in SGPRs
    uint32_t vlan_tag_word;                 // GROW: the 4 pushed bytes {TPID, TCI} as a LE dword
    uint32_t mtu;                           // SZ_MTU: --mtu; tile t's output at input offset - tcut[t]
    const long long *tcut;
    uint32_t *grow_bad;                     // SZ_MTU / SZ_FUZZ: a tile whose cut differs from tcut's
    const uint32_t *fz_state;               // SZ_FUZZ: each record's RNG state (te_fuzz_states)
    uint32_t fz_factor;                     // SZ_FUZZ: --fuzz-factor
    uint32_t stream;                        // nontemporal span loads and output stores (a batch larger
                                            // than the 256 MiB Infinity Cache: read once, written once)
    // window mode (te_wave_tiles<..., WIN>: the record discovery fused into the edit)
    uint64_t win_len;                       // image bytes (records end here)
    uint64_t win_entry;                     // image offset of the first record, or, when set,
    const uint64_t *win_entry_ptr;          //   *win_entry_ptr - win_entry_sub (a pipeline chunk:
    uint64_t win_entry_sub;                 //   where the previous chunk's chain ended)
    uint64_t win_base, win_limit;           // the window grid's origin; records starting at limit on
                                            //   are not the image's
    uint32_t nwin;
    uint64_t *w_entry, *w_exit;             // per window: where the chain enters and leaves it
    uint32_t *w_flags;                      // per window: IDX_STOP / IDX_ERROR / IDX_END / IDX_TRIM, WIN_F_EDIT
    uint32_t *win_bad;                      // the verdict (te_win_check): bit 0 the chain, bit 1 a
                                            //   record left to the exact path; zeroed here
    unsigned long long *win_tot;            // the chain's end (te_win_check); zeroed here
};

// the window's partly valid dword for fl::phase_a: packet bytes [4k - 2, caplen), k =
// (caplen + 2) / 4, read from the unedited image at window start wa (packet offset -2);
// 0 when caplen + 2 is a multiple of 4 or the dword lies past the window
// (window_part_n: over a window of NWX dwords)
template <int NWX>
__device__ __forceinline__ uint32_t window_part_n(const uint8_t *S, uint32_t wa, uint32_t caplen) {
    const uint32_t t = caplen + 2, k = t >> 2, nb = t & 3u;
    const uint32_t q = (wa & ~3u) + 4u * umin32(k, NWX - 1);
    const uint32_t e0 = *(const uint32_t *)(S + q), e1 = *(const uint32_t *)(S + q + 4);
    const uint32_t keep = (nb != 0 && k < (uint32_t)NWX) ? ((1u << (8 * nb)) - 1u) : 0u;
    return __builtin_amdgcn_alignbyte(e1, e0, wa & 3u) & keep;
}
__device__ __forceinline__ uint32_t window_part(const uint8_t *S, uint32_t wa, uint32_t caplen) {
    return window_part_n<fl::NW>(S, wa, caplen);
}

// one's-complement sum of the LE 16-bit words (absolute pairing) of bytes [b0, b1) of chunk c
__device__ __forceinline__ uint32_t chunk_part(const uint8_t *S, uint32_t c, int b0, int b1) {
    const uint4 v = *(const uint4 *)(S + 16 * c);
    return fl::wsum(v.x & fl::bmask(b0, b1)) + fl::wsum(v.y & fl::bmask(b0 - 4, b1 - 4)) +
           fl::wsum(v.z & fl::bmask(b0 - 8, b1 - 8)) + fl::wsum(v.w & fl::bmask(b0 - 12, b1 - 12));
}

// folded sum of LDS bytes [x, y) (x < y, absolute pairing) from the chunk prefix P
__device__ __forceinline__ uint32_t lds_range_sum(const uint8_t *S, const uint32_t *P, uint32_t x, uint32_t y) {
    const uint32_t cx = x >> 4, cy = y >> 4;
    unsigned long long sum;
    if (cx == cy) {
        sum = chunk_part(S, cx, (int)(x & 15), (int)(y & 15));
    } else {
        sum = chunk_part(S, cx, (int)(x & 15), 16);
        sum += P[cy] - P[cx + 1];
        if (y & 15) sum += chunk_part(S, cy, 0, (int)(y & 15));
    }
    return fold16(sum);
}

__global__ void __launch_bounds__(FKB, TE_FK_MIN_BLOCKS) te_fast_tiles(FastArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t S[FK_LDS];
    __shared__ __attribute__((aligned(16))) uint32_t P[FK_NCH + 1];
    __shared__ __attribute__((aligned(16))) te_dev_cfg_t cfg;
    __shared__ uint32_t wsums[FKB / 64];
    // per tile: bit 0 some packet deferred, bit 1 some packet needs the chunk prefix.  Two
    // slots by iteration parity: the other slot is cleared only after the fill barrier, when
    // every thread has read it (a deferred tile leaves the loop without an end barrier)
    __shared__ uint32_t tflags[2];
    const int tid = threadIdx.x;
    {
        const uint32_t *src = (const uint32_t *)a.cfg;
        uint32_t *dst = (uint32_t *)&cfg;
        for (int i = tid; i < (int)(sizeof(te_dev_cfg_t) / 4); i += FKB) dst[i] = src[i];
    }
    if (blockIdx.x == 0) {
        if (tid < 4) a.ws_zero[tid] = 0;  // the generic kernel's err words and ticket
        if (tid == 4) *a.list_cnt_next = 0;
    }
    const bool swp = a.in_swapped != 0;
    const bool explicit_dir = a.fixed_dir >= 0;
    g_cu8 *gin = (g_cu8 *)a.in;
    g_u8 *gout = (g_u8 *)a.out;
    const TE_AS_GLOBAL uint16_t *lut = (const TE_AS_GLOBAL uint16_t *)a.portlut;
    unsigned long long c_pkts = 0, c_bytes = 0, c_edited = 0;
    __syncthreads();

    constexpr int K = (TE_FK_TILE_BYTES / 16 + FKB - 1) / FKB + 1;  // 16-byte chunks per lane per tile
    static_assert(K <= 8, "FK_EACH covers 8 chunk registers");
    // this tile's chunks in flight, in named registers (an array indexed in a loop that
    // the compiler may re-roll ends up in scratch)
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
#define FK_EACH(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define FK_LD(k)                                                        \
    if constexpr (k < K) {                                              \
        const uint32_t c = umin32((uint32_t)tid + k * FKB, nc_ - 1u);   \
        v##k = *(g_cu4 *)(gin + a0_ + ((uint64_t)c << 4));              \
    }
// unconditional (a huge tile loads its first chunk K times): the vector-memory
// count is then the same on every path and the waits stay partial
#define FK_ISSUE(tl)                                                                              \
    {                                                                                             \
        const uint64_t a0_ = (tl).span_off & ~15ull;                                              \
        const uint32_t nc_ = (tl).scratch_off == TE_NO_SCRATCH                                    \
                                 ? (uint32_t)(((tl).span_off + (tl).span_len - a0_ + 15) >> 4)   \
                                 : 1u;                                                            \
        FK_EACH(FK_LD)                                                                            \
        rel_next = pkt_rel[(tl).first_pkt + umin32((uint32_t)tid, (tl).npkt - 1u)];                \
    }
#define FK_ST(k)                                                                              \
    if constexpr (k < K) { /* branch-free: lanes past the span write a dummy slot */         \
        const uint32_t c = (uint32_t)tid + k * FKB;                                           \
        *(uint4 *)(S + (c < nchunks ? LDS_FRONT + (c << 4) : FK_LDS - 16)) = v##k;            \
    }
    const uint32_t G = gridDim.x;
    // descriptors through the constant address space: scalar loads (lgkmcnt), so
    // fetching one never waits on the vector loads in flight
    const TE_AS_CONST te_tile_t *tiles = (const TE_AS_CONST te_tile_t *)a.tiles;
    const TE_AS_CONST uint16_t *pkt_rel = (const TE_AS_CONST uint16_t *)a.pkt_rel;
    te_tile_t cur, nxt;
    uint32_t rel_next = 0;  // this lane's record offset in the tile whose chunks are in flight
    if (blockIdx.x < a.n_tiles) {
        cur = tiles[blockIdx.x];
        FK_ISSUE(cur);
    }
    if (blockIdx.x + G < a.n_tiles) nxt = tiles[blockIdx.x + G];
#if TE_FK_STAMPS
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, last_ = __builtin_amdgcn_s_memtime(), ntl = 0;
#endif
    if (tid == 0) tflags[0] = tflags[1] = 0;
    __syncthreads();
    uint32_t slot = 0;
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += G, slot ^= 1u) {
        FK_STAMP(0)  // loop overhead / previous iteration tail
        const te_tile_t tile = cur;
        const bool huge = tile.scratch_off != TE_NO_SCRATCH;
        const uint32_t npkt = tile.npkt;
        const uint64_t G0 = tile.span_off, A0 = G0 & ~15ull;
        const uint32_t my_rel = rel_next;
        const uint32_t img = LDS_FRONT + (uint32_t)(G0 - A0) + tile.span_len;  // LDS bytes in use
        {  // ---- span -> LDS (also for a huge tile: harmless, and keeps the waits partial) ----
            const uint32_t nchunks = huge ? 0u : (uint32_t)((G0 + tile.span_len - A0 + 15) >> 4);
            FK_EACH(FK_ST)
        }
        __syncthreads();
        if (tid == 0) tflags[slot ^ 1u] = 0;
#if TE_FK_PREFETCH
        // the next tile's loads fly while this one is edited and stored
        cur = nxt;
        if (t + G < a.n_tiles) FK_ISSUE(cur);
        if (t + 2 * G < a.n_tiles) nxt = tiles[t + 2 * G];
#endif
        if (huge) {  // a record larger than a tile: generic lane
            if (tid == 0) a.tile_list[atomicAdd(a.list_cnt, 1u)] = t;
#if !TE_FK_PREFETCH
            cur = nxt;
            if (t + G < a.n_tiles) FK_ISSUE(cur);
            if (t + 2 * G < a.n_tiles) nxt = tiles[t + 2 * G];
#endif
            continue;
        }
#if !TE_FK_PREFETCH
        cur = nxt;
        if (t + 2 * G < a.n_tiles) nxt = tiles[t + 2 * G];
#endif

        FK_STAMP(1)  // fill LDS (waits for the prefetched chunks) + barrier + next prefetch issue
        // ---- phase A: one lane per packet ----
        const uint32_t r0 = LDS_FRONT + (uint32_t)(G0 - A0) + my_rel;  // record header in S
        const uint32_t p = r0 + 16;                                    // packet data in S
        const uint32_t wa = p - 2;                                     // window start (packet offset -2)
        uint32_t H[fl::NW];
        uint32_t d0 = 0, caplen = 0, len = 0;
        fl::State st;
        st.do_l4 = st.tail = false;
        st.dirty = 0;
        bool ok = true, nosend = false;
        if (tid < (int)npkt) {
            {  // caplen, len: three aligned dword reads + funnel shifts (not eight byte reads)
                const uint32_t h8 = r0 + 8, ha = h8 & ~3u, hs = h8 & 3u;
                const uint32_t w0 = *(const uint32_t *)(S + ha), w1 = *(const uint32_t *)(S + ha + 4),
                               w2 = *(const uint32_t *)(S + ha + 8);
                caplen = __builtin_amdgcn_alignbyte(w1, w0, hs);
                len = __builtin_amdgcn_alignbyte(w2, w1, hs);
                if (swp) {
                    caplen = bswap32(caplen);
                    len = bswap32(len);
                }
            }
            const uint64_t pktno = a.pkt_base + tile.first_pkt + tid;
            int dir = TE_DIR_C2S;
            if (explicit_dir) {
                dir = a.fixed_dir;
            } else if (a.dirbits) {  // check_cache (src/common/cache.c:321-354)
                const uint64_t idx = pktno >> 2;
                const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
                const uint8_t b = idx < a.dirbits_len ? a.dirbits[idx] : 0;
                dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
            }
            if (dir == TE_DIR_NOSEND && !explicit_dir) {  // tcprewrite.c:314-315: written unedited
                nosend = true;
            } else {
                // 8-byte aligned ds_read_b64 pairs (half the bank conflicts of dword reads), then
                // a dword select and a byte funnel shift align the window to packet offset -2
                const uint32_t A8 = wa & ~7u, s8 = wa & 7u, sh = s8 & 3u;
                uint32_t d[fl::NW + 2];
#pragma unroll
                for (int j = 0; j < fl::NW + 2; j += 2) {
                    const uint2 q = *(const uint2 *)(S + A8 + 4 * j);
                    d[j] = q.x;
                    d[j + 1] = q.y;
                }
                const uint32_t mh = s8 >= 4 ? 0xffffffffu : 0u;  // bitwise select: an index ternary
                uint32_t e[fl::NW + 1];                             // would move d[] to scratch
#pragma unroll
                for (int j = 0; j <= fl::NW; ++j) e[j] = (d[j + 1] & mh) | (d[j] & ~mh);
#pragma unroll
                for (int i = 0; i < fl::NW; ++i) H[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sh);
                d0 = e[0];
                ok = fl::phase_a<TE_FF_ALL>(H, caplen, len, window_part(S, wa, caplen), dir, cfg, fl::knobs_of(cfg),
                                            a.v6_ok != 0, lut, st);
            }
        }
        {
            const uint32_t f = (ok ? 0u : 1u) | (st.tail ? 2u : 0u);
            if (f) atomicOr(&tflags[slot], f);
        }
        __syncthreads();
        const uint32_t tf = tflags[slot];
        FK_STAMP(2)  // phase A + its barrier
        if (tf & 1u) {  // a packet for the generic lane: it redoes this tile
            if (tid == 0) a.tile_list[atomicAdd(a.list_cnt, 1u)] = t;
#if !TE_FK_PREFETCH
            if (t + G < a.n_tiles) FK_ISSUE(cur);
#endif
            continue;
        }

        // ---- chunk prefix for L4 bytes past the windows (large packets only) ----
        if (tf & 2u) {
            const uint32_t nch = (img + 15) >> 4;
            for (uint32_t c = tid; c < nch; c += FKB) {
                const uint4 v = *(const uint4 *)(S + 16 * c);
                P[c] = fl::wsum(v.x) + fl::wsum(v.y) + fl::wsum(v.z) + fl::wsum(v.w);
            }
            __syncthreads();
            uint32_t loc[FK_Q], tot = 0;
#pragma unroll
            for (int k = 0; k < FK_Q; ++k) {
                const uint32_t c = (uint32_t)tid * FK_Q + k;
                const uint32_t v = c < nch ? P[c] : 0u;
                loc[k] = tot;
                tot += v;
            }
            uint32_t total;
            const uint32_t base = block_exscan<FKB>(tot, wsums, total);
#pragma unroll
            for (int k = 0; k < FK_Q; ++k) {
                const uint32_t c = (uint32_t)tid * FK_Q + k;
                if (c < nch) P[c] = base + loc[k];
            }
            if (tid == 0) P[nch] = total;
            __syncthreads();
        }

        FK_STAMP(3)  // chunk prefix
        // ---- phase B + write-back of the dwords phase A touched ----
        if (tid < (int)npkt) {
            if (!nosend) {
                uint32_t tail = 0;
                if (st.tail) {
                    tail = lds_range_sum(S, P, p + fl::WEND, p + st.end);
                    if (p & 1) tail = fl::swap16(tail);  // absolute -> packet-relative pairing
                }
                fl::phase_b(H, st, tail);
                const uint32_t A = wa & ~3u, sh = wa & 3u;
                // LDS dword j holds window bytes from H[j-1] and H[j] (from H[j] alone when aligned)
                const uint32_t need = st.dirty | (sh ? (st.dirty << 1) : 0u);
#pragma unroll
                for (int j = 0; j < fl::NW; ++j) {
                    if (!((need >> j) & 1u)) continue;
                    const uint32_t prev = j ? H[j - 1] : (d0 << (8 * (4 - sh)));
                    const uint32_t v = sh ? __builtin_amdgcn_alignbyte(H[j], prev, 4 - sh) : H[j];
                    const int rel = (int)(A + 4 * j) - (int)p;  // packet offset of the dword's first byte
                    uint8_t *q = S + A + 4 * j;
                    if (rel + 4 <= (int)caplen) {
                        *(uint32_t *)q = v;
                    } else {
#pragma unroll
                        for (int b = 0; b < 3; ++b)
                            if (rel + b < (int)caplen) q[b] = (uint8_t)(v >> (8 * b));
                    }
                }
            }
            if (swp || a.in_nsec) {  // header in host order, microseconds
                uint8_t *rec = S + r0;
                uint32_t ts_sec = ld_hdr32(rec, swp), ts_frac = ld_hdr32(rec + 4, swp);
                if (a.in_nsec) ts_frac /= 1000;
                st32(rec, ts_sec);
                st32(rec + 4, ts_frac);
                st32(rec + 8, caplen);
                st32(rec + 12, len);
            }
            ((g_u8 *)a.status)[tile.first_pkt + tid] = nosend ? (uint8_t)TE_ST_NOSEND : (uint8_t)0;
        }
        const uint32_t n_nosend = __syncthreads_count(nosend);
        FK_STAMP(4)  // phase B + write-back + status + barrier

        // ---- span LDS -> HBM at its input offset: output chunk C is LDS chunk
        //      C - G0 + LDS_FRONT + (G0 - A0), i.e. 16-byte aligned on both sides ----
        {
            const uint64_t Gs = a.out_base + (G0 - a.rec0), Ge = Gs + tile.span_len, C0 = Gs & ~15ull;
            const uint32_t nchunks = (uint32_t)((Ge - C0 + 15) >> 4);
            const int64_t lds_of_out = (int64_t)(LDS_FRONT + (uint32_t)(G0 - A0)) - (int64_t)Gs;
            // all LDS reads first (one LDS latency), then the stores
            constexpr int KS = (TE_FK_TILE_BYTES / 16 + 2 + FKB - 1) / FKB;
            uint4 w[KS];
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                const uint32_t c = umin32((uint32_t)tid + k * FKB, nchunks - 1u);
                w[k] = *(const uint4 *)(S + (int64_t)(C0 + ((uint64_t)c << 4)) + lds_of_out);
            }
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                const uint32_t c = (uint32_t)tid + k * FKB;
                if (c < nchunks) {
                    const uint64_t C = C0 + ((uint64_t)c << 4);
                    const int b0 = C < Gs ? (int)(Gs - C) : 0;
                    const int b1 = (C + 16 > Ge) ? (int)(Ge - C) : 16;
                    const uint4 v = w[k];
                    g_u8 *dst = gout + C;
                    if (b0 == 0 && b1 == 16) {
                        *(g_u4 *)dst = v;
                    } else {
#pragma unroll
                        for (int b = 0; b < 16; ++b) {
                            if (b >= b0 && b < b1) {
                                const uint32_t x = b < 4 ? v.x : (b < 8 ? v.y : (b < 12 ? v.z : v.w));
                                dst[b] = (uint8_t)(x >> (8 * (b & 3)));
                            }
                        }
                    }
                }
            }
        }
        FK_STAMP(5)  // stores issued
        c_pkts += npkt;
        c_bytes += tile.span_len;
        c_edited += npkt - n_nosend;
#if TE_FK_STAMPS
        ++ntl;
#endif
#if !TE_FK_PREFETCH
        if (t + G < a.n_tiles) FK_ISSUE(cur);
#endif
        __syncthreads();
    }
#undef FK_ISSUE
#undef FK_LD
#undef FK_ST
#undef FK_EACH
#if TE_FK_STAMPS
    if (tid == 0 && (blockIdx.x == 0 || blockIdx.x == 1 || blockIdx.x == 137 || blockIdx.x == gridDim.x - 1))
        printf("stamps block %u tiles %llu: top %llu fill %llu phaseA %llu prefix %llu phaseB %llu store %llu\n",
               blockIdx.x, ntl, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5]);
#endif
    if (tid < TE_CNT__N) {  // fire-and-forget adds of the block's totals
        unsigned long long v = 0;
        if (tid == TE_CNT_PACKETS || tid == TE_CNT_WRITTEN) v = c_pkts;
        else if (tid == TE_CNT_BYTES_IN || tid == TE_CNT_BYTES_OUT) v = c_bytes;
        else if (tid == TE_CNT_EDITED) v = c_edited;
        if (v) atomicAdd(&a.counters[tid], v);
    }
}

// ===========================================================================
// te_wave_tiles: the fast lane with one WAVE per tile -- at most 64
// consecutive records whose span (plus the next record's header) fits
// TE_WK_TILE_BYTES.  The waves of a block share only the cfg copy.  Each owns
// an LDS image and a chunk-prefix array, streams its own span in, edits and
// stores it, and never meets a workgroup barrier inside the tile loop: one
// wave's LDS accesses are performed in order, so its write -> read hand-offs
// need none.  Tiles are dealt statically (wave w of the grid takes w, w + W,
// w + 2W, ...), and the next tile's span is in flight in registers while the
// current one is edited and stored.
//
// Output (static offsets: output byte q sits at input byte q + out_base -
// rec0, a multiple of 16): a tile stores the 16-byte chunks that START inside
// its span, and its leading bytes (span start to the next 16-byte boundary)
// one byte per lane.  Its last chunk carries at most 15 bytes of the next
// tile, all inside that tile's first record header, which both waves compute
// alike (for big-endian / nanosecond input the image then holds that whole
// header and converts it too).  So no chunk needs bytes of two waves merged.
// A tile the lane cannot finish (a deferred packet, or a record larger than
// the image) stores nothing and is listed; the generic kernel, next on the
// stream, writes its whole span byte-exactly.
//
// Every path that writes the next span into LDS has issued the same stores
// since that span's loads (lanes past the span repeat a chunk or byte of it
// instead of skipping the store), so the compiler's wait there can be partial:
// it waits for the loads, not for this tile's stores.
// ===========================================================================
#ifndef TE_WK_MIN_BLOCKS
#define TE_WK_MIN_BLOCKS 4  // blocks per CU (= waves per SIMD at 256 threads): 128 VGPRs
#endif
// the lean instances (no option group that reads the cfg tables: no LDS copy of them)
// fit one more block per CU -- 5 waves per SIMD at <= 102 VGPRs, 31 KiB of LDS a block
#ifndef TE_WK_LEAN_BLOCKS
#define TE_WK_LEAN_BLOCKS 5
#endif
// The lean instances also cut tiles to TE_WK_LEAN_TILE_BYTES: 63 C2 records (80 B) fill five
// 16-byte chunk loads per lane exactly, where 64 records and the next header need six.
#ifndef TE_WK_SMALL_BLOCKS
#define TE_WK_SMALL_BLOCKS TE_WK_LEAN_BLOCKS  // (the TE_FF_SMALL instances)
#endif
#ifndef TE_WK_LEAN_TILE_BYTES
#define TE_WK_LEAN_TILE_BYTES 5120
#endif
// The lean size-preserving instances of the exact path (tiles from the host index) cut tiles
// to TE_WK_BIG_TILE_BYTES at 4 blocks/CU: a 1,514-byte record's tile then holds five records,
// not three (C5 0.585 -> 0.627 of peak, C2 and c2x10 unchanged: 64 records cap a C2 tile
// either way; A/B on one box, tools/gpu_abbench.sh).  Window mode and the sized
// instances keep TE_WK_LEAN_TILE_BYTES (their LDS budgets hold 4 and 5 blocks/CU).
#ifndef TE_WK_BIG_TILE_BYTES
#define TE_WK_BIG_TILE_BYTES 8192
#endif
#ifndef TE_WK_BIG_BLOCKS
#define TE_WK_BIG_BLOCKS TE_WK_MIN_BLOCKS
#endif
// (TE_FF_SMALL instances keep TE_WK_LEAN_TILE_BYTES at 5 blocks/CU: a batch of C2's 80-byte
// records fills 63 of them into 5 KiB, so the 8 KiB image buys nothing but a block per CU --
// C2 0.626 -> 0.678 of peak, seed 0.685 -> 0.70, A/B on one box, round 6; the cfg-reading
// ones TE_WK_TILE_BYTES at 4 blocks/CU: 1M x 64 B under --pnat --portmap 0.50 -> 0.58)
// the size-preserving exact-path instances that read the cfg: their tile budget and blocks/CU
// (8 KiB at 3 blocks/CU: an IMIX tile holds ~22 records, not ~16, and the per-tile phases
//  edit a third more records a pass -- C3 0.607 -> 0.623, hdr 0.624 -> 0.645, macseed
//  0.623 -> 0.641 of peak, A/B on one box, round 6; 6 KiB at 4 blocks before)
#ifndef TE_WK_READS_TILE_BYTES
#define TE_WK_READS_TILE_BYTES 8192
#endif
#ifndef TE_WK_READS_BLOCKS
#define TE_WK_READS_BLOCKS 3
#endif
// the static +-4 instances (VLAN push / pop, --efcs: wk_store_sized) likewise: C4 0.564 ->
// 0.581, vdel 0.589 -> 0.595, efcs 0.591 -> 0.595 (their chunk map sized by the budget);
// 9 KiB (51,840 B of LDS a block, 3 blocks in 160 KiB): C4 0.584 -> 0.586-0.596, vdel +0.2 %
// (10 KiB does not fit 3 blocks; 9 KiB for the size-preserving cfg instances: C3, hdr -1 %)
#ifndef TE_WK_SIZED_TILE_BYTES
#define TE_WK_SIZED_TILE_BYTES 9216
#endif
#ifndef TE_WK_SIZED_BLOCKS
#define TE_WK_SIZED_BLOCKS 3
#endif
// the per-record cut instances (--mtu-trunc, --fuzz-seed: wk_store_mtu): their tile budget
// for the lean and the cfg-reading instances
// (8 KiB at 3 blocks/CU, a map of 16 entries a lane: mtu 0.547 -> 0.587, fz 0.365 -> 0.412 of
//  peak, A/B on one box, round 6; the lean 5 KiB / cfg 6 KiB budgets before -- 0 restores them;
//  9 KiB, still 3 blocks in 160 KiB: mtu 0.585 -> 0.604, fz 0.431 -> 0.460)
#ifndef TE_WK_CUT_TILE_BYTES
#define TE_WK_CUT_TILE_BYTES 9216
#endif
#ifndef TE_WK_CUT_BLOCKS
#define TE_WK_CUT_BLOCKS 3  // (0: as the other lean / cfg instances; --fuzz-seed: TE_WK_FUZZ_BLOCKS)
#endif
#ifndef TE_WK_SIZED_LEAN_TILE_BYTES
#define TE_WK_SIZED_LEAN_TILE_BYTES TE_WK_SIZED_TILE_BYTES
#endif
#ifndef TE_WK_SIZED_LEAN_BLOCKS
#define TE_WK_SIZED_LEAN_BLOCKS TE_WK_SIZED_BLOCKS
#endif
template <uint32_t F, int SZ = 0, bool WIN = false>
struct WkCfg {  // does instance F read te_dev_cfg_t (its LDS copy); its occupancy target and tile budget
    static constexpr bool reads = (F & (TE_FF_MAC | TE_FF_PORTMAP | TE_FF_RWIP | TE_FF_HDR)) != 0;
    static constexpr bool big = !reads && SZ == 0 && !WIN && !(F & TE_FF_SMALL);
    static constexpr bool rbig = reads && SZ == 0 && !WIN && !(F & TE_FF_SMALL);
    static constexpr bool sized = SZ == TE_SZ_GROW || SZ == TE_SZ_VDEL || SZ == TE_SZ_EFCS;
    static constexpr int blocks = rbig    ? TE_WK_READS_BLOCKS
                                  : sized ? (reads ? TE_WK_SIZED_BLOCKS : TE_WK_SIZED_LEAN_BLOCKS)
                                  : SZ == TE_SZ_MTU && TE_WK_CUT_BLOCKS ? TE_WK_CUT_BLOCKS
                                  : big ? TE_WK_BIG_BLOCKS
                                  : reads ? TE_WK_MIN_BLOCKS
                                  : (F & TE_FF_SMALL) && SZ == 0 && !WIN ? TE_WK_SMALL_BLOCKS : TE_WK_LEAN_BLOCKS;
    static constexpr bool cut = SZ == TE_SZ_MTU || SZ == TE_SZ_FUZZ;
    static constexpr int tile = rbig    ? TE_WK_READS_TILE_BYTES
                                : sized ? (reads ? TE_WK_SIZED_TILE_BYTES : TE_WK_SIZED_LEAN_TILE_BYTES)
                                : cut && TE_WK_CUT_TILE_BYTES ? TE_WK_CUT_TILE_BYTES
                                : reads ? TE_WK_TILE_BYTES : big ? TE_WK_BIG_TILE_BYTES : TE_WK_LEAN_TILE_BYTES;
};
#ifndef TE_WK_STORE_BARRIER
#define TE_WK_STORE_BARRIER 1
#endif
// the size-preserving store fills the next tile's span into LDS between its LDS reads and
// its global stores (0: after the stores, as before round 6)
#ifndef TE_WK_FILL_EARLY
#define TE_WK_FILL_EARLY 1
#endif
// and for the per-record cut stores (wk_store_mtu: --mtu-trunc, --fuzz-seed; A/B: mtu 1.8 %
// slower, fz even -- off)
#ifndef TE_WK_CUT_FILL_EARLY
#define TE_WK_CUT_FILL_EARLY 0
#endif
// the same for the static +4 store (wk_store_sized, VLAN push: C4 0.596 -> 0.600, A/B)
#ifndef TE_WK_SIZED_FILL_EARLY
#define TE_WK_SIZED_FILL_EARLY 1
#endif
#ifndef TE_WK_LANE_OPAQUE
#define TE_WK_LANE_OPAQUE 1
#endif
constexpr int WKB = TE_WK_BLOCK;
constexpr int WK_NW = WKB / 64;                          // waves (tiles in flight) per block
// per tile budget TB: 16-byte chunks per lane, the LDS image (+ phase-A window overrun),
// the chunk prefix (+ total)
constexpr int wk_kl(int tb) { return tb / 16 / 64; }
constexpr int wk_img(int tb) { return LDS_FRONT + tb + 128; }
constexpr int wk_nch(int tb) { return tb / 16 + 2; }
// window mode: sub-window bytes per lane and lookback lanes of the discovery (te_window.hpp),
// the bytes a window's last record may reach past the staged window (a longer one is left to
// the exact path), and the window image: front pad, the staged window, that tail, slack
#ifndef TE_WIN_S
#define TE_WIN_S 80  // bytes a lane scans: a window is 64 of them
#endif
#ifndef TE_WIN_OL
#define TE_WIN_OL 2  // of which the first TE_WIN_OL lanes' are the previous window's
#endif
constexpr int WIN_S = TE_WIN_S, WIN_OL = TE_WIN_OL;
constexpr int WIN_W = 64 * WIN_S, WIN_WN = WIN_W - WIN_OL * WIN_S;
#ifndef TE_WIN_TAIL
#define TE_WIN_TAIL 2048
#endif
constexpr int WIN_TAIL = TE_WIN_TAIL;
// staged with the window past its end + 16 (five 1 KiB wave loads in all): the last
// record reaching past the window is in LDS without a second, dependent load unless longer
#ifndef TE_WIN_PRE
#define TE_WIN_PRE (-1)  // (A/B: the bytes staged past a window's end + 16; -1: fill the last 1 KiB load)
#endif
constexpr int WIN_PRE = TE_WIN_PRE >= 0 ? TE_WIN_PRE : 1024 * ((WIN_W + 48 + 900 + 1023) / 1024) - WIN_W - 48;
static_assert(WIN_PRE >= 0 && WIN_PRE <= WIN_TAIL, "window pre-staging within the tail room");
constexpr int WIN_IMG = LDS_FRONT + WIN_W + 48 + WIN_TAIL + 128;
constexpr int WIN_REL = 4 * WIN_S + 1;
// a window's flags word (w_flags): the discovery's chain stops (IDX_*), and this bit when
// the edit left one of its records to the exact path -- te_win_check turns either into the
// batch's verdict, so nothing writes the verdict words during the window kernel, which
// zeroes them itself (no fill launch a run)
constexpr uint32_t WIN_F_EDIT = 0x100u;
static_assert((WIN_F_EDIT & (IDX_STOP | IDX_ERROR | IDX_END | IDX_TRIM)) == 0, "a flag bit of its own");
static_assert(WIN_W + 48 + WIN_TAIL < 65536, "record offsets from a window's start fit 16 bits");
static_assert(WIN_IMG % 16 == 0, "16-byte aligned window images");
static_assert(TE_WK_TILE_BYTES % 1024 == 0 && wk_kl(TE_WK_TILE_BYTES) <= 16, "whole chunks per lane, <= 16 registers");
static_assert(TE_WK_BIG_TILE_BYTES % 1024 == 0 && wk_kl(TE_WK_BIG_TILE_BYTES) <= 16, "big tile budget");
// the sized stores (VLAN push / pop, --efcs) map a tile's output chunks 8 or 16 entries a
// lane (wk_store_sized: round 6, after 7 and 8 KiB builds of the 512-entry map wrote wrong
// C4 bytes in round 5): at most 1,024 chunks
static_assert(TE_WK_SIZED_TILE_BYTES % 1024 == 0 && (TE_WK_SIZED_TILE_BYTES + 256) / 16 + 1 <= 1024,
              "the sized stores' chunk map: at most 1,024 entries");
static_assert(TE_WK_LEAN_TILE_BYTES % 1024 == 0 && wk_kl(TE_WK_LEAN_TILE_BYTES) <= 16, "lean tile budget");
static_assert(wk_img(TE_WK_TILE_BYTES) % 16 == 0 && wk_img(TE_WK_LEAN_TILE_BYTES) % 16 == 0, "16-byte aligned images");

// TE_WK_STAMPS builds (diagnostics only): s_memtime per phase, summed per wave,
// printed by a few waves at exit
#if TE_WK_STAMPS
#define WK_STAMP(i)                                                        \
    {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                 \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
        __builtin_amdgcn_sched_barrier(0);                                 \
        ph[i] += now_ - last_;                                             \
        last_ = now_;                                                      \
    }
#else
#define WK_STAMP(i)
#endif

__device__ __forceinline__ bool wk_solo(const te_tile_t &tl, uint32_t tb) {
    // (the last test: a span the image cannot hold never reaches the lane, whatever the cut)
    return (tl.flags & TE_TILE_SOLO) != 0 || tl.scratch_off != TE_NO_SCRATCH ||
           (uint32_t)(tl.span_off & 15) + tl.span_len + 16u > tb;
}

// size-changing instances (SZ): the one length change every record takes
enum : int {
    SZ_NONE = TE_SZ_NONE,
    SZ_GROW = TE_SZ_GROW,
    SZ_VDEL = TE_SZ_VDEL,
    SZ_EFCS = TE_SZ_EFCS,
    SZ_MTU = TE_SZ_MTU,
    SZ_FUZZ = TE_SZ_FUZZ
};

// caplen and len of the record header at LDS byte h (any alignment) + delta: the VLAN
// push's +4 (tcpedit.c:112-113), the VLAN pop's or --efcs's -4 (tcpedit.c:78-84)
__device__ __forceinline__ void hdr_add4(uint8_t *S, uint32_t h, uint32_t delta) {
    const uint32_t h8 = h + 8, al = h8 & ~3u, s8 = 8u * (h8 & 3u);
    uint32_t *w = (uint32_t *)(S + al);
    const uint32_t q0 = w[0], q1 = w[1], q2 = w[2];
    const uint32_t cap = __builtin_amdgcn_alignbyte(q1, q0, h8 & 3u) + delta;
    const uint32_t len = __builtin_amdgcn_alignbyte(q2, q1, h8 & 3u) + delta;
    if (s8 == 0) {
        w[0] = cap;
        w[1] = len;
    } else {
        const uint32_t lo = (1u << s8) - 1u;  // bytes of q0 below the caplen field
        w[0] = (q0 & lo) | (cap << s8);
        w[1] = (cap >> (32u - s8)) | (len << s8);
        w[2] = (q2 & ~lo) | (len >> (32u - s8));
    }
}

// caplen = len = v in the record header at LDS byte h (any alignment): --mtu-trunc's cut
// (edit_packet.c:599)
__device__ __forceinline__ void hdr_put(uint8_t *S, uint32_t h, uint32_t v) {
    const uint32_t h8 = h + 8, al = h8 & ~3u, s8 = 8u * (h8 & 3u);
    uint32_t *w = (uint32_t *)(S + al);
    if (s8 == 0) {
        w[0] = v;
        w[1] = v;
    } else {
        const uint32_t lo = (1u << s8) - 1u, q0 = w[0], q2 = w[2];
        w[0] = (q0 & lo) | (v << s8);
        w[1] = (v >> (32u - s8)) | (v << s8);
        w[2] = (q2 & ~lo) | (v >> (32u - s8));
    }
}

// inclusive wave scans and the previous lane's value: wave_dpp.hpp (call them where every
// lane of the wave is active -- tests/test_dpp.py)
// Size-changing stores (GROW: a 4-byte tag pushed into every record; SHRINK: 4 bytes
// dropped from every record).  Record j's change sits at tile-relative input offset D_j,
// and consecutive changes are >= 58 bytes apart, so a 16-byte output chunk meets at most
// one.  Per output chunk c one 16-bit word of the chunk map K says
//   bits 0-6   m: the changes wholly before the chunk (its bytes come from the input 4 m
//              bytes back under GROW, on under SHRINK), and
//   bits 7-11  where change m meets the chunk: 0 not at all, else 4 + its offset from the
//              chunk start (GROW: -3..15, the tag may start in the previous chunk;
//              SHRINK: 1..15)
// built from one mark per change and a prefix max, so each chunk's store is one map read
// and one batch of five dword reads -- no dependent lookups.
// LDS hand-off between lanes of one wave: its LDS accesses are performed in order, but
// the compiler, reasoning per lane, would forward a lane's own store to its later load of
// the same address across other lanes' stores to it (it did: the chunk map's prefix read
// came back as the zeros this lane had written, without the other lanes' marks)
#ifndef WK_SKIP_TOUCHED
#define WK_SKIP_TOUCHED 1
#endif
#ifndef WK_SIZED_STREAM
#define WK_SIZED_STREAM 0
#endif
#ifndef WK_MTU_STREAM
#define WK_MTU_STREAM 0  // SZ_MTU: nontemporal chunk stores on batches past the Infinity Cache
#endif
#ifndef WK_PLAIN_STREAM
#define WK_PLAIN_STREAM 1
#endif
#define WK_LANES_SYNC() asm volatile("" ::: "memory")

// (NE: map entries a lane, 8 for tiles up to 6 KiB -- 512 entries -- 16 past them)
template <int NE>
__device__ __forceinline__ void wk_chunk_map(uint32_t *P, uint32_t nown, uint32_t o0, uint32_t X, bool on,
                                             bool grow, int lane) {
    static_assert(NE == 8 || NE == 16, "whole uint4s of entries a lane");
    uint16_t *K = (uint16_t *)P;  // 64 NE entries
#pragma unroll
    for (int h = 0; h < NE / 8; ++h) *(uint4 *)(K + NE * lane + 8 * h) = make_uint4(0, 0, 0, 0);
    // the first chunk that change j lies wholly before (GROW: the tag [X, X + 4) has ended;
    // SHRINK: the boundary X is at or before the chunk start)
    const uint32_t wb = grow ? X + 4u : X;
    if (on) {
        const uint32_t cj = (wb - o0 + 15u) >> 4;
        if (cj < nown) K[cj] = (uint16_t)(lane + 1);
    }
    WK_LANES_SYNC();
    {  // prefix max over K, NE entries a lane
        uint32_t e[NE];
#pragma unroll
        for (int h = 0; h < NE / 8; ++h) {
            const uint4 q = *(const uint4 *)(K + NE * lane + 8 * h);
            e[8 * h + 0] = q.x & 0xffffu, e[8 * h + 1] = q.x >> 16, e[8 * h + 2] = q.y & 0xffffu;
            e[8 * h + 3] = q.y >> 16, e[8 * h + 4] = q.z & 0xffffu, e[8 * h + 5] = q.z >> 16;
            e[8 * h + 6] = q.w & 0xffffu, e[8 * h + 7] = q.w >> 16;
        }
#pragma unroll
        for (int i = 1; i < NE; ++i) e[i] = max(e[i], e[i - 1]);
        const uint32_t excl = wave_prev(wave_scan_max(e[NE - 1]));
#pragma unroll
        for (int i = 0; i < NE; ++i) e[i] = max(e[i], excl);
#pragma unroll
        for (int h = 0; h < NE / 8; ++h)
            *(uint4 *)(K + NE * lane + 8 * h) =
                make_uint4(e[8 * h] | (e[8 * h + 1] << 16), e[8 * h + 2] | (e[8 * h + 3] << 16),
                           e[8 * h + 4] | (e[8 * h + 5] << 16), e[8 * h + 6] | (e[8 * h + 7] << 16));
    }
    WK_LANES_SYNC();
    // the chunks change j meets (whose m is j): where
    if (on) {
        const uint32_t c1 = (X - o0) >> 4, t1 = X - o0 - 16u * c1;  // the chunk X lies in
        if (grow) {
            if (c1 < nown) K[c1] = (uint16_t)(lane | ((t1 + 4u) << 7));
            if (t1 > 12u && c1 + 1 < nown) K[c1 + 1] = (uint16_t)(lane | ((t1 - 12u) << 7));  // its tail
        } else if (t1 != 0 && c1 < nown) {
            K[c1] = (uint16_t)(lane | ((t1 + 4u) << 7));
        }
    }
    WK_LANES_SYNC();
}

// the 16 output bytes of a chunk that change m meets, from the 20 input bytes dd starting
// 4 (m + 1) bytes back (GROW) / 4 m bytes on (SHRINK); tc: the change's offset from the
// chunk start (GROW: the tag's, -3..15; SHRINK: the boundary's, 1..15)
__device__ __forceinline__ void mix_grow(const uint32_t (&dd)[5], int tc, uint32_t tag, uint32_t (&w)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int t = tc - 4 * i;  // the tag's start relative to this dword
        const uint32_t before = dd[i + 1], after = dd[i];
        const int tp = t < 0 ? 0 : (t > 3 ? 3 : t), tn = t > -1 ? 1 : (t < -3 ? 3 : -t);
        const uint32_t mp = (1u << (8 * tp)) - 1u, mn = (1u << (8 * (4 - tn))) - 1u;
        const uint32_t vp = (before & mp) | ((tag << (8 * tp)) & ~mp);   // tag starts in this dword
        const uint32_t vn = ((tag >> (8 * tn)) & mn) | (after & ~mn);    // tag started tn bytes earlier
        w[i] = t >= 4 ? before : (t <= -4 ? after : (t >= 0 ? vp : vn));
    }
}
__device__ __forceinline__ void mix_shrink(const uint32_t (&dd)[5], int tc, uint32_t (&w)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int t = tc - 4 * i;  // the boundary relative to this dword
        const uint32_t mk = (1u << (8 * (t < 1 ? 1 : (t > 3 ? 3 : t)))) - 1u;
        const uint32_t mixed = (dd[i] & mk) | (dd[i + 1] & ~mk);
        w[i] = t >= 4 ? dd[i] : (t <= 0 ? dd[i + 1] : mixed);
    }
}

__device__ __forceinline__ void wk_put16(g_u8 *gout, uint64_t at, const uint32_t (&w)[4], bool stream) {
    if (stream)
        __builtin_nontemporal_store((u32x4){w[0], w[1], w[2], w[3]}, (g_v4 *)(gout + at));
    else
        *(g_u4 *)(gout + at) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Size-changing stores.  Every chunk that no change meets is a plain 16-byte copy of the
// input 4 m bytes back (GROW) / on (SHRINK): one pass over the tile's chunks stores them
// with no byte mixing; then each record's lane builds the one or two chunks its own change
// meets and stores them over the first pass's bytes (one wave's stores to an address are
// performed in order).  (Mixing in the chunk pass costs every chunk the VALU work
// of the few that need it: C4 spent a third of its kernel there.)
// (TB: the tile budget; the output chunks of a tile number <= (TB + 256) / 16 + 1: NK rounds
//  of 64, a map of NE entries a lane)
// pre_store (TE_WK_SIZED_FILL_EARLY): called after every LDS read of the image, before the
// first global store (the step's next span into LDS there); returns whether it ran
template <bool GROW, int TB, typename PRE>
__device__ __forceinline__ bool wk_store_sized(const uint8_t *S, uint32_t *P, g_u8 *gout, uint64_t OS,
                                               uint32_t span_len, uint32_t npkt, uint32_t g0, uint32_t X,
                                               bool on, uint32_t tag, int lane, bool stream, PRE &&pre_store) {
    constexpr int NK = ((TB + 256) / 16 + 1 + 63) / 64, NE = NK <= 8 ? 8 : 16;
    static_assert(NE * 64 * 2 <= wk_nch(TB) * 4, "the chunk map fits the chunk-prefix array");
    const uint64_t OE = GROW ? OS + span_len + 4ull * npkt : OS + span_len - 4ull * npkt;
    const uint64_t C0 = (OS + 15) & ~15ull;
    const uint32_t o0 = (uint32_t)(C0 - OS);
    const uint32_t nown = (uint32_t)((((OE + 15) & ~15ull) - C0) >> 4);  // <= 64 NK
    wk_chunk_map<NE>(P, nown, o0, X, on, GROW, lane);
    const uint16_t *K = (const uint16_t *)P;
    const uint8_t *img = S + LDS_FRONT + g0;  // input byte x of the tile
    // every read in flight before the first store (a store under its own branch would
    // otherwise pull its reads in after it and wait them out one chunk at a time)
    uint32_t kv[NK], w[NK][4];
#pragma unroll
    for (int k = 0; k < NK; ++k) kv[k] = K[umin32((uint32_t)lane + 64u * k, nown - 1u)];
#pragma unroll
    for (int k = 0; k < NK; ++k) {  // lanes past the output repeat its last chunk (same bytes)
        const uint32_t cc = umin32((uint32_t)lane + 64u * k, nown - 1u);
        const uint32_t m = kv[k] & 127u;
        const uint32_t o = o0 + 16u * cc;
        const uint32_t *D = (const uint32_t *)(GROW ? img + o - 4u * m : img + o + 4u * m);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[k][i] = D[i];
    }
    if constexpr (TE_WK_SIZED_FILL_EARLY && GROW) {
    // every read of the image (the change chunks' and the leading byte's too) before the
    // next span overwrites it, then the stores: the wait for that span's loads no longer
    // covers this tile's stores (GROW only: C4 +0.6 %; --efcs ran 2.4 % slower so)
    const uint32_t c1 = (X - o0) >> 4, t1 = X - o0 - 16u * c1;
    uint32_t w2[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t o = o0 + 16u * umin32(c1 + (uint32_t)h, nown - 1u);
        const uint32_t *D = (const uint32_t *)(GROW ? img + o - 4u * (uint32_t)lane - 4u : img + o + 4u * (uint32_t)lane);
        const uint32_t dd[5] = {D[0], D[1], D[2], D[3], D[4]};
        const int tc = (int)t1 - 16 * h;
        if constexpr (GROW) mix_grow(dd, tc, tag, w2[h]);
        else mix_shrink(dd, tc, w2[h]);
    }
    const uint64_t q = (uint32_t)lane < o0 ? OS + (uint32_t)lane : C0;  // others repeat byte C0
    const uint8_t lead = img[(uint32_t)(q - OS)];
    WK_LANES_SYNC();
    const bool filled = pre_store();
#if WK_SKIP_TOUCHED
#pragma unroll
    for (int k = 0; k < NK; ++k)
        if ((kv[k] >> 7) == 0u) wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nown - 1u), w[k], stream);
#else
#pragma unroll
    for (int k = 0; k < NK; ++k) wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nown - 1u), w[k], stream);
#endif
    if (on && (GROW || t1 != 0) && c1 < nown) wk_put16(gout, C0 + 16ull * c1, w2[0], stream);
    if (on && GROW && t1 > 12u && c1 + 1 < nown) wk_put16(gout, C0 + 16ull * (c1 + 1), w2[1], stream);
    gout[q] = lead;
    return filled;
    } else {
    WK_LANES_SYNC();
    // chunks no change meets are stored here; the few a change meets are stored below, by
    // the same wave (skipping them here measured 0.6% faster on C4 than storing every chunk
    // and overwriting; WK_SKIP_TOUCHED=0 restores the unconditional form)
#if WK_SKIP_TOUCHED
#pragma unroll
    for (int k = 0; k < NK; ++k)
        if ((kv[k] >> 7) == 0u) wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nown - 1u), w[k], stream);
#else
#pragma unroll
    for (int k = 0; k < NK; ++k) wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nown - 1u), w[k], stream);
#endif
    // the chunks this lane's change meets: both built on every lane (reads in flight
    // together), stored where they exist
    {
        const uint32_t j = (uint32_t)lane, c1 = (X - o0) >> 4, t1 = X - o0 - 16u * c1;
        uint32_t w2[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t o = o0 + 16u * umin32(c1 + (uint32_t)h, nown - 1u);
            const uint32_t *D = (const uint32_t *)(GROW ? img + o - 4u * j - 4u : img + o + 4u * j);
            const uint32_t dd[5] = {D[0], D[1], D[2], D[3], D[4]};
            const int tc = (int)t1 - 16 * h;
            if constexpr (GROW) mix_grow(dd, tc, tag, w2[h]);
            else mix_shrink(dd, tc, w2[h]);
        }
        WK_LANES_SYNC();
        if (on && (GROW || t1 != 0) && c1 < nown) wk_put16(gout, C0 + 16ull * c1, w2[0], stream);
        if (on && GROW && t1 > 12u && c1 + 1 < nown) wk_put16(gout, C0 + 16ull * (c1 + 1), w2[1], stream);
    }
    // the leading bytes (output start to the first 16-byte boundary: before any change)
    const uint64_t q = (uint32_t)lane < o0 ? OS + (uint32_t)lane : C0;  // others repeat byte C0
    gout[q] = img[(uint32_t)(q - OS)];
    (void)pre_store;
    return false;
    }
}

// --mtu-trunc and --fuzz-seed stores (SZ_MTU, SZ_FUZZ).  A kept record j keeps its first
// 16 + caplen'_j bytes (keep false: a record that keeps nothing, a fuzz DROP); the kept
// records sit back to back from the tile's output offset OS, record j at tile-relative
// output offset op_j (a wave scan of the kept sizes) and input offset rel_j.  The kept
// records are numbered 0.. in order (ballot + popcount) and only they take part: per output
// chunk the map K names the kept record holding its first byte (one mark per record + a
// prefix max, as wk_chunk_map); bit 15 marks a chunk a record starts inside of.  Pass 1
// stores every other chunk as one unaligned 16-byte LDS read of its record (the cut moves
// records by any byte count: five dwords, four funnel shifts).  Pass 2: each record's lane
// builds the chunk it starts inside of from the previous kept record's tail and its own
// head.  The leading bytes (OS up to the first 16-byte boundary) and the trailing ones (the
// last boundary up to the tile's output end) go a byte a lane, so a tile writes only its
// own output bytes: the next tile's first record header, which the last chunk would carry,
// is not known here.  A kept record is >= 17 bytes, so a chunk meets at most two of them,
// and the leading / trailing bytes lie in at most two.
// P: K in u16 [0, 512), the kept-record table {rel_j | op_j << 16} in u32 [256, 320).
// (The previous record's {rel, op} came from wave_prev DPP shifts once, under the EXEC mask
// of the pass-2 branch: wrong bytes -- wave_dpp.hpp, DESIGN.md 4.13.  It is read from T.)
// DROPS (SZ_FUZZ): records may keep nothing and a record may be as short as 17 bytes, so
// the kept ones are numbered apart from their lanes and a tile may have no whole chunk;
// without it (SZ_MTU) the kept records are lanes [0, npkt) and each is >= 50 bytes.
// (NE: map entries a lane -- 8, or 16 for tiles past 8 KiB of output chunks -- the record
//  table T then starts at u32 32 NE: P holds >= 32 NE + 64 words, wk_mtu_nch)
// pre_store (TE_WK_CUT_FILL_EARLY): as wk_store_sized's
template <int NK, bool DROPS, int NE, typename PRE>
__device__ __forceinline__ bool wk_store_mtu(const uint8_t *S, uint32_t ib, uint32_t *P, g_u8 *gout, uint64_t OS,
                                             uint32_t out_len, uint32_t npkt, uint32_t my_rel, uint32_t my_op,
                                             bool keep, int lane, bool stream, PRE &&pre_store) {
    static_assert(NE == 8 || NE == 16, "whole uint4s of entries a lane");
    static_assert(NK <= NE, "the map covers the full chunks");
    if (DROPS && out_len == 0) return false;  // (wave-uniform: every record dropped)
    uint32_t ci = (uint32_t)lane, nk = npkt;  // this record's kept number; the kept records
    if constexpr (DROPS) {
        const unsigned long long km = __ballot(keep);
        ci = (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
        nk = (uint32_t)__popcll(km);
    }
    const uint64_t C0 = (OS + 15) & ~15ull;
    const uint32_t o0 = (uint32_t)(C0 - OS);
    const uint32_t nfull = (out_len - o0) >> 4;  // (out_len >= 17 > o0; MTU: nfull >= 2)
    uint16_t *K = (uint16_t *)P;
    uint32_t *T = P + 32 * NE;
#pragma unroll
    for (int h = 0; h < NE / 8; ++h) *(uint4 *)(K + NE * lane + 8 * h) = make_uint4(0, 0, 0, 0);
    if (keep) T[ci] = my_rel | (my_op << 16);
    WK_LANES_SYNC();
    if (keep) {  // the first chunk starting at or after op_j (the first kept record: chunk 0)
        const uint32_t cj = my_op <= o0 ? 0u : (my_op - o0 + 15u) >> 4;
        if (cj <= nfull) K[cj] = (uint16_t)(ci + 1);
    }
    WK_LANES_SYNC();
    {  // prefix max over K, NE entries a lane
        uint32_t e[NE];
#pragma unroll
        for (int h = 0; h < NE / 8; ++h) {
            const uint4 q = *(const uint4 *)(K + NE * lane + 8 * h);
            e[8 * h + 0] = q.x & 0xffffu, e[8 * h + 1] = q.x >> 16, e[8 * h + 2] = q.y & 0xffffu;
            e[8 * h + 3] = q.y >> 16, e[8 * h + 4] = q.z & 0xffffu, e[8 * h + 5] = q.z >> 16;
            e[8 * h + 6] = q.w & 0xffffu, e[8 * h + 7] = q.w >> 16;
        }
#pragma unroll
        for (int i = 1; i < NE; ++i) e[i] = max(e[i], e[i - 1]);
        const uint32_t excl = wave_prev(wave_scan_max(e[NE - 1]));
#pragma unroll
        for (int i = 0; i < NE; ++i) e[i] = max(e[i], excl);
#pragma unroll
        for (int h = 0; h < NE / 8; ++h)
            *(uint4 *)(K + NE * lane + 8 * h) =
                make_uint4(e[8 * h] | (e[8 * h + 1] << 16), e[8 * h + 2] | (e[8 * h + 3] << 16),
                           e[8 * h + 4] | (e[8 * h + 5] << 16), e[8 * h + 6] | (e[8 * h + 7] << 16));
    }
    WK_LANES_SYNC();
    // kept record j > 0 starting inside a chunk: K there already names kept record j - 1 (value j)
    const uint32_t x = (keep && ci > 0) ? my_op - o0 : 16u, c1 = x >> 4, t1 = x & 15u;
    if (t1 != 0 && c1 < nfull) K[c1] = (uint16_t)(ci | 0x8000);
    WK_LANES_SYNC();
    if constexpr (TE_WK_CUT_FILL_EARLY) {
        // every read of the image first (pass 1's, pass 2's, the trailing and leading bytes'),
        // then the next span into LDS, then the stores
        const bool p1 = !DROPS || nfull;  // (wave-uniform)
        uint32_t kv[NK], w[NK][4];
        if (p1) {
#pragma unroll
            for (int k = 0; k < NK; ++k) kv[k] = K[umin32((uint32_t)lane + 64u * k, nfull - 1u)];
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const uint32_t cc = umin32((uint32_t)lane + 64u * k, nfull - 1u);
                const uint32_t e = T[(kv[k] & 0x7fu) - 1u];
                const uint4 v = read16(S, ib + (e & 0xffffu) + o0 + 16u * cc - (e >> 16));
                w[k][0] = v.x;
                w[k][1] = v.y;
                w[k][2] = v.z;
                w[k][3] = v.w;
            }
        }
        const uint32_t ep = T[ci > 0 ? ci - 1 : 0], prel = ep & 0xffffu, pop = ep >> 16;
        const uint32_t q = o0 + 16u * c1;
        const bool p2 = t1 != 0 && c1 < nfull;
        const uint4 va = read16(S, p2 ? ib + prel + (q - pop) : ib);
        const uint4 vb = read16(S, p2 ? ib + my_rel - t1 : ib);
        const uint32_t A[4] = {va.x, va.y, va.z, va.w}, B[4] = {vb.x, vb.y, vb.z, vb.w};
        uint32_t m[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t mk = fl::bmask(0, (int)t1 - 4 * i);
            m[i] = (A[i] & mk) | (B[i] & ~mk);
        }
        const uint32_t q0t = o0 + 16u * nfull, ntr = out_len - q0t;
        const uint32_t qb = q0t + umin32((uint32_t)lane, ntr ? ntr - 1u : 0u);
        const uint32_t j = (K[nfull] & 0x7fu) - 1u;
        const uint32_t e1 = T[umin32(j + 1u, nk - 1u)];
        const uint32_t e = (j + 1u < nk && qb >= (e1 >> 16)) ? e1 : T[j];
        const uint8_t tv = S[ib + (e & 0xffffu) + qb - (e >> 16)];
        const uint32_t ll = (uint32_t)lane < o0 ? (uint32_t)lane : 0u;
        const uint8_t lv = S[ib + (DROPS ? T[0] & 0xffffu : 0u) + ll];
        WK_LANES_SYNC();
        const bool filled = pre_store();
        if (p1) {
#pragma unroll
            for (int k = 0; k < NK; ++k)
                if ((kv[k] >> 15) == 0u)
                    wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nfull - 1u), w[k], stream);
        }
        if (p2) wk_put16(gout, C0 + 16ull * c1, m, stream);
        if ((uint32_t)lane < ntr) gout[OS + qb] = tv;
        if ((uint32_t)lane < o0) gout[OS + (uint32_t)lane] = lv;
        return filled;
    }
    if (!DROPS || nfull) {  // (wave-uniform)
        uint32_t kv[NK], w[NK][4];
#pragma unroll
        for (int k = 0; k < NK; ++k) kv[k] = K[umin32((uint32_t)lane + 64u * k, nfull - 1u)];
#pragma unroll
        for (int k = 0; k < NK; ++k) {  // lanes past the output repeat its last full chunk
            const uint32_t cc = umin32((uint32_t)lane + 64u * k, nfull - 1u);
            const uint32_t e = T[(kv[k] & 0x7fu) - 1u];
            const uint4 v = read16(S, ib + (e & 0xffffu) + o0 + 16u * cc - (e >> 16));
            w[k][0] = v.x;
            w[k][1] = v.y;
            w[k][2] = v.z;
            w[k][3] = v.w;
        }
        WK_LANES_SYNC();
#pragma unroll
        for (int k = 0; k < NK; ++k)
            if ((kv[k] >> 15) == 0u)
                wk_put16(gout, C0 + 16ull * umin32((uint32_t)lane + 64u * k, nfull - 1u), w[k], stream);
    }
    {  // pass 2: the chunk kept record j starts inside of (the previous one's {rel, op} from T)
        const uint32_t ep = T[ci > 0 ? ci - 1 : 0], prel = ep & 0xffffu, pop = ep >> 16;
        const uint32_t q = o0 + 16u * c1;
        const bool p2 = t1 != 0 && c1 < nfull;  // (the first kept record, the others: x = 16, t1 = 0)
        // (the lanes that store nothing read the image start: every address stays in it)
        const uint4 va = read16(S, p2 ? ib + prel + (q - pop) : ib);
        const uint4 vb = read16(S, p2 ? ib + my_rel - t1 : ib);
        const uint32_t A[4] = {va.x, va.y, va.z, va.w}, B[4] = {vb.x, vb.y, vb.z, vb.w};
        uint32_t m[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t mk = fl::bmask(0, (int)t1 - 4 * i);
            m[i] = (A[i] & mk) | (B[i] & ~mk);
        }
        WK_LANES_SYNC();
        if (p2) wk_put16(gout, C0 + 16ull * c1, m, stream);
    }
    {  // the trailing bytes [o0 + 16 nfull, out_len), a byte a lane
        const uint32_t q0t = o0 + 16u * nfull, ntr = out_len - q0t;
        const uint32_t qb = q0t + umin32((uint32_t)lane, ntr ? ntr - 1u : 0u);
        const uint32_t j = (K[nfull] & 0x7fu) - 1u;
        const uint32_t e1 = T[umin32(j + 1u, nk - 1u)];
        const uint32_t e = (j + 1u < nk && qb >= (e1 >> 16)) ? e1 : T[j];
        const uint8_t v = S[ib + (e & 0xffffu) + qb - (e >> 16)];
        if ((uint32_t)lane < ntr) gout[OS + qb] = v;
    }
    // the leading bytes: the first kept record's (op 0; MTU: record 0, rel 0)
    if ((uint32_t)lane < o0) gout[OS + (uint32_t)lane] = S[ib + (DROPS ? T[0] & 0xffffu : 0u) + (uint32_t)lane];
    (void)pre_store;
    return false;
}

// big-endian / nanosecond input: a record header in host order and microseconds
__device__ __forceinline__ void conv_hdr(uint8_t *rec, bool swp, bool nsec) {
    const uint32_t ts_sec = ld_hdr32(rec, swp), cl = ld_hdr32(rec + 8, swp), ln = ld_hdr32(rec + 12, swp);
    uint32_t ts_frac = ld_hdr32(rec + 4, swp);
    if (nsec) ts_frac /= 1000;
    st32(rec, ts_sec);
    st32(rec + 4, ts_frac);
    st32(rec + 8, cl);
    st32(rec + 12, ln);
}

// the window of a record whose VLAN tag the pop removes, as the popped packet sees it:
// packet' bytes [-2, 12) are the input's, [12, 78) the input's [16, 82).  HX: the input
// window [-2, 82) (NW + 1 dwords)
__device__ __forceinline__ void vdel_view(uint32_t (&H)[fl::NW], const uint32_t (&HX)[fl::NW + 1]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) H[i] = HX[i];
    H[3] = (HX[3] & 0xffffu) | (HX[4] & 0xffff0000u);
#pragma unroll
    for (int i = 4; i < fl::NW; ++i) H[i] = HX[i + 1];
}

// WIN: window mode -- no tile list: each wave takes byte windows of the image, finds the
// records starting in its window (te_window.hpp), cuts them into tiles as the host would and
// edits them in place in the staged window (size-preserving instances, native-order
// microsecond input, no tcpprep cache).  Each window leaves where the chain enters and leaves
// it for te_win_check; a record the lane cannot finish sets win_bad, and the caller then runs
// the exact path (index + tiles) instead.
template <uint32_t F, int DEPTH, int SZ, bool WIN = false>
#ifndef TE_WIN_PREFETCH
#define TE_WIN_PREFETCH 0
#endif
#ifndef TE_WIN_BLOCKS
#define TE_WIN_BLOCKS TE_WK_MIN_BLOCKS  // window mode: blocks per CU (its VGPR budget)
#endif
#ifndef TE_WIN_LEAN_BLOCKS
#define TE_WIN_LEAN_BLOCKS TE_WIN_BLOCKS  // ... for the lean instances (no cfg copy in LDS)
#endif
// (SZ_FUZZ: TE_WK_FUZZ_BLOCKS per CU, one fewer with the address maps -- at the lean
//  instances' 5 / the others' 4 the fuzz step's registers spill)
#ifndef TE_WK_FUZZ_BLOCKS
#define TE_WK_FUZZ_BLOCKS (TE_WK_CUT_TILE_BYTES > 6144 ? 3 : TE_WK_MIN_BLOCKS)
#endif
__global__ void __launch_bounds__(WKB, WIN              ? (WkCfg<F>::reads ? TE_WIN_BLOCKS : TE_WIN_LEAN_BLOCKS)
                                       : SZ == SZ_FUZZ ? (WkCfg<F>::reads && TE_WK_CUT_TILE_BYTES <= 6144 ? TE_WK_FUZZ_BLOCKS - 1
                                                                                                    : TE_WK_FUZZ_BLOCKS)
                                       : (DEPTH == 2 && (WkCfg<F, SZ, WIN>::blocks) > TE_WK_MIN_BLOCKS)
                                                       ? TE_WK_MIN_BLOCKS  // (two spans in flight: >= 128 VGPRs)
                                                       : (WkCfg<F, SZ, WIN>::blocks)) te_wave_tiles(FastArgs a) {
    constexpr int TB = WkCfg<F, SZ, WIN>::tile, WK_KL = wk_kl(TB), WK_IMG = WIN ? WIN_IMG : wk_img(TB);
    // (--mtu-trunc / --fuzz-seed stores: a map of MTU_NE entries a lane and a 64-word record
    //  table after it, in the chunk-prefix array)
    constexpr int MTU_NE = WK_KL + 1 <= 8 ? 8 : 16;
    constexpr int WK_NCH = (SZ == SZ_MTU || SZ == SZ_FUZZ) && 32 * MTU_NE + 64 > wk_nch(TB) ? 32 * MTU_NE + 64
                                                                                         : wk_nch(TB);
    static_assert(!WIN || SZ == SZ_NONE, "window mode: size-preserving instances");
    constexpr bool GROW = SZ == SZ_GROW, VDEL = SZ == SZ_VDEL, EFCS = SZ == SZ_EFCS, SHRINK = VDEL || EFCS;
    constexpr bool MTU = SZ == SZ_MTU, FUZZ = SZ == SZ_FUZZ;
    // VLAN pop: the window reaches 4 input bytes further (the packet' view skips the tag)
    constexpr int XW = VDEL ? 1 : 0;
    __shared__ __attribute__((aligned(16))) uint8_t SB[WK_NW][WK_IMG];
    __shared__ __attribute__((aligned(16))) uint32_t PB[WK_NW][WK_NCH];
    // per-run tables: copied only by instances whose option groups read them
    __shared__ __attribute__((aligned(16))) uint8_t cfg_raw[WkCfg<F>::reads ? sizeof(te_dev_cfg_t) : 16];
    const te_dev_cfg_t &cfg = *(const te_dev_cfg_t *)cfg_raw;
    __shared__ unsigned long long red[WK_NW][6];
    __shared__ uint16_t RELB[WIN ? WK_NW : 1][WIN ? WIN_REL : 1];  // window mode: record offsets
    const int tid = threadIdx.x;
    int lane = tid & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
    if constexpr (WkCfg<F>::reads) {
        const uint32_t *src = (const uint32_t *)a.cfg;
        uint32_t *dst = (uint32_t *)cfg_raw;
        for (int i = tid; i < (int)(sizeof(te_dev_cfg_t) / 4); i += WKB) dst[i] = src[i];
    }
    if (blockIdx.x == 0) {
        if (tid < 4) a.ws_zero[tid] = 0;  // the generic kernel's err words and ticket
        if (tid == 4) *a.list_cnt_next = 0;
        if (tid >= 8 && tid < 8 + TE_CNT__N) a.counters_next[tid - 8] = 0;  // (the generic pass may not run)
    }
    uint8_t *S = SB[wid];
    uint32_t *P = PB[wid];
    const bool swp = a.in_swapped != 0, nsec = a.in_nsec != 0, conv = swp || nsec;
    const bool explicit_dir = a.fixed_dir >= 0;
    // the next record's header rides along (conversion; GROW / SHRINK: its caplen/len +- 4)
    // (--mtu-trunc, --fuzz-seed: a tile stores only its own output bytes, so nothing rides along)
    const uint32_t extra = (conv || (SZ != SZ_NONE && !MTU && !FUZZ)) ? 16u : 0u;
    g_cu8 *gin = (g_cu8 *)a.in;
    g_u8 *gout = (g_u8 *)a.out + ((int64_t)a.out_base - (int64_t)a.rec0);
    const TE_AS_GLOBAL uint16_t *lut = (const TE_AS_GLOBAL uint16_t *)a.portlut;
    const TE_AS_CONST te_tile_t *tiles = (const TE_AS_CONST te_tile_t *)a.tiles;
    const TE_AS_CONST uint16_t *pkt_rel = (const TE_AS_CONST uint16_t *)a.pkt_rel;
    const fl::Knobs kn{a.seed_sw, a.seed_on != 0, a.skip_bcast != 0};
    const bool stream = a.stream != 0;  // wave-uniform (an SGPR): a scalar branch per batch of loads/stores
    __syncthreads();

    // a tile in flight: its descriptor, its chunks in named registers, and this lane's
    // record offset and tcpprep cache byte
    struct Span {
        te_tile_t tl;
        uint4 v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11, v12, v13, v14, v15;
        uint32_t rel, dirb;
        bool dirv;     // (the cache byte exists: idx < dirbits_len)
        uint32_t fzs;  // FUZZ: the record's RNG state
    };
#define WK_EACH(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
    const uint32_t W = gridDim.x * WK_NW;
    const uint32_t w0 = blockIdx.x * WK_NW + wid;
    const uint32_t n_tiles = a.n_tiles;
    unsigned long long c_pkts = 0, c_bytes = 0, c_edited = 0, c_cut = 0, c_drop = 0, c_soft = 0;
#if TE_WK_STAMPS
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, last_ = __builtin_amdgcn_s_memtime(), ntl = 0;
    unsigned long long fph[5] = {0, 0, 0, 0, 0};  // (window mode: inside the record discovery)
#endif

    // loads of a tile's span (its chunks, record offsets and cache bytes) into R
    auto issue = [&](Span &R, const te_tile_t &tl) __attribute__((always_inline)) {
        R.tl = tl;
        const uint64_t a0_ = tl.span_off & ~15ull;
        const uint32_t nc_ = wk_solo(tl, TB) ? 1u : (uint32_t)((tl.span_off + tl.span_len + extra - a0_ + 15) >> 4);
#define WK_LD(k)                                                                              \
    if constexpr (k < WK_KL) {                                                                \
        const uint32_t c = umin32((uint32_t)lane + k * 64u, nc_ - 1u);                        \
        if (stream) {                                                                         \
            const u32x4 nv = __builtin_nontemporal_load((g_cv4 *)(gin + a0_ + ((uint64_t)c << 4))); \
            R.v##k = make_uint4(nv.x, nv.y, nv.z, nv.w);                                      \
        } else {                                                                              \
            R.v##k = *(g_cu4 *)(gin + a0_ + ((uint64_t)c << 4));                              \
        }                                                                                     \
    }
        WK_EACH(WK_LD)
#undef WK_LD
        const uint32_t k_ = tl.first_pkt + umin32((uint32_t)lane, tl.npkt - 1u);
        R.rel = pkt_rel[k_];
        R.fzs = FUZZ ? a.fz_state[k_] : 0u;
        if (a.dirbits) {  // in flight with the span (no consumer here: its wait would drain the span)
            const uint64_t ix_ = (a.pkt_base + k_) >> 2;
            R.dirb = a.dirbits[ix_ < a.dirbits_len ? ix_ : 0];
            R.dirv = ix_ < a.dirbits_len;
        } else {
            R.dirb = 0;
            R.dirv = false;
        }
    };
    // R's chunks -> the LDS image, the whole image unconditionally: chunks past the span
    // land past it (never read as data).  Waits for R's loads only.
    auto fill = [&](const Span &R) __attribute__((always_inline)) {
#define WK_ST(k) \
    if constexpr (k < WK_KL) *(uint4 *)(S + LDS_FRONT + (((uint32_t)lane + k * 64u) << 4)) = R.v##k;
        WK_EACH(WK_ST)
#undef WK_ST
        // the span's per-lane loads (issued after its chunks) are taken here too, on every path
        // that fills: otherwise the loop's copy of them waits at the back edge, where the paths
        // merge with different store counts, for every store of the tile just done (vmcnt(0))
        asm volatile("" ::"v"(R.rel), "v"(R.dirb), "v"(R.fzs));
    };
    // edit and store tile t, whose span is in the LDS image; a tile the lane cannot
    // finish is listed for the generic lane and stores nothing
    // pre_store(): called by the size-preserving store between its LDS reads and its global
    // stores -- the step puts the next tile's span into LDS there (TE_WK_FILL_EARLY), so the
    // wait for that span's loads no longer covers this tile's stores (vmcnt counts both, in
    // issue order); returns whether it ran
    auto edit = [&](const uint32_t t, const te_tile_t &tile, const uint32_t my_rel, const uint32_t my_dirb,
                    const bool my_dirv, const uint32_t my_fzs, auto &&pre_store) __attribute__((always_inline)) -> bool {
            const uint32_t npkt = tile.npkt;
            const uint64_t G0 = tile.span_off, A0 = G0 & ~15ull, E = G0 + tile.span_len;
            const uint32_t g0 = (uint32_t)(G0 - A0);
            if (wk_solo(tile, TB)) {  // a record larger than the image: the generic lane
                if (WIN) {
                    if (lane == 0) atomicOr(&a.w_flags[t], WIN_F_EDIT);
                } else if (lane == 0) {
                    a.tile_list[atomicAdd(a.list_cnt, 1u)] = t;
                }
                return false;
            }

            // ---- phase A: one lane per packet ----
            const uint32_t r0 = LDS_FRONT + g0 + my_rel;  // record header in S
            const uint32_t p = r0 + 16;                   // packet data in S
            const uint32_t wa = p - 2;                    // window start (packet offset -2)
            const bool on = lane < (int)npkt;
            // every lane reads a header and a window (lanes past npkt: the tile's last
            // record's), so H has one definition and no lane-dependent merge copies
            uint32_t caplen, len;
            {  // caplen, len: three aligned dword reads + funnel shifts
                const uint32_t h8 = r0 + 8, ha = h8 & ~3u, hs = h8 & 3u;
                const uint32_t q0 = *(const uint32_t *)(S + ha), q1 = *(const uint32_t *)(S + ha + 4),
                               q2 = *(const uint32_t *)(S + ha + 8);
                caplen = __builtin_amdgcn_alignbyte(q1, q0, hs);
                len = __builtin_amdgcn_alignbyte(q2, q1, hs);
                if (swp) {
                    caplen = bswap32(caplen);
                    len = bswap32(len);
                }
            }
            // --fuzz-seed (SZ_FUZZ): fuzzing() for a record its draw picks (tcpedit.c:250-258,
            // fuzzing.c:80-199), before the window is read.  The lane plans it for the header
            // shape phase A takes (Ethernet II, IPv4 IHL 5 or IPv6, TCP or UDP: a packet of
            // another shape sends the tile to the generic lane, which plans it itself).  A byte
            // run lands in the image (a changed record is checksummed from scratch: fuzzing()'s
            // 1 is a needtorecalc); a cut (DROP / REDUCE) fails the second decode (a soft error,
            // tcpedit.c:95-99), so the record is written unedited at its first nl bytes.
            bool fz_cut = false, fz_recalc = false;
            uint32_t fz_nl = 0;
            if constexpr (FUZZ) {
                uint32_t s_ = my_fzs;
                const uint32_t r = tcpr_random_dev(s_);
                if (on && r % a.fz_factor == 0u) {
                    const bool v6 = S[p + 12] == 0x86u && S[p + 13] == 0xDDu;
                    const uint32_t proto = v6 ? S[p + 20] : S[p + 23];
                    const int l3 = v6 ? 54 : 34, l4h = proto == 6u ? 20 : 8;
                    const FzPlan f = fuzz_plan_l4(r, l3 + l4h, l3 - l4h, caplen, len);
                    // the run [from, from + n) (<= 15 bytes), cut at caplen (past it lies the
                    // reference's buffer, never output, and here the next record), as five
                    // aligned dwords read together and written back under byte masks (a byte
                    // loop waited out the LDS latency per byte); records' runs are >= 58 bytes
                    // apart, so no other lane writes these dwords now
                    const uint32_t lo = p + (uint32_t)f.from, hi = p + umin32((uint32_t)(f.from + f.n), caplen);
                    if (f.n > 0 && hi > lo) {
                        const uint32_t a4 = lo & ~3u;
                        uint32_t q[5];
#pragma unroll
                        for (int k = 0; k < 5; ++k) q[k] = *(const uint32_t *)(S + a4 + 4 * k);
                        const uint32_t xv = 0x01010101u * f.x;
#pragma unroll
                        for (int k = 0; k < 5; ++k) {
                            const uint32_t m = fl::bmask((int)lo - (int)(a4 + 4 * k), (int)hi - (int)(a4 + 4 * k));
                            const uint32_t v = f.how == 0 ? 0u : f.how == 1 ? 0xffffffffu : (q[k] ^ xv);
                            if (m) *(uint32_t *)(S + a4 + 4 * k) = (q[k] & ~m) | (v & m);
                        }
                    }
                    fz_cut = f.cut;
                    fz_recalc = f.ret != 0 && !f.cut;
                    fz_nl = f.nl;
                }
                WK_LANES_SYNC();  // the window reads below see every lane's run
            }
            // 21 dword-aligned reads (paired into ds_read2_b32) and a funnel shift align
            // the window to packet offset -2; each H[i] can take d[i]'s register
            uint32_t H[fl::NW], d0;
            // SHRINK: the packet's caplen/len after the pop or the FCS strip (a record whose
            // caplen != len keeps its caplen under --efcs: phase A defers it)
            // MTU: untrunc_packet's cut (edit_packet.c:596-611): a packet longer than l2len + mtu
            // keeps that many bytes (l2len 14 on this lane; phase A classifies the packet as
            // captured and checksums the cut one)
            const bool mcut = MTU && len > a.mtu + 14u;
            const uint32_t ecap = SHRINK ? caplen - 4u : (mcut ? a.mtu + 14u : caplen);
            const uint32_t elen = SHRINK ? len - 4u : (mcut ? a.mtu + 14u : len);
            bool tagged = true;  // VDEL: a single 802.1Q / 802.1ad / QinQ-TPID tag at offset 12
            {
                const uint32_t A4 = wa & ~3u, sh = wa & 3u;
                uint32_t d[fl::NW + 1 + XW];
#pragma unroll
                for (int j = 0; j <= fl::NW + XW; ++j) d[j] = *(const uint32_t *)(S + A4 + 4 * j);
                if constexpr (VDEL) {
                    uint32_t HX[fl::NW + 1];
#pragma unroll
                    for (int i = 0; i <= fl::NW; ++i) HX[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
                    const uint32_t tpid = HX[3] >> 16;  // raw LE: 0x8100, 0x88a8, 0x9100
                    tagged = tpid == 0x0081u || tpid == 0xa888u || tpid == 0x0091u;
                    vdel_view(H, HX);
                } else {
#pragma unroll
                    for (int i = 0; i < fl::NW; ++i) H[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
                }
                d0 = d[0];
            }
            // the partly valid dword: packet' dword k' is input dword k' + 1 under the pop
            const uint32_t part = VDEL ? window_part_n<fl::NW + 1>(S, wa, caplen) : window_part(S, wa, ecap);
            int dir = TE_DIR_C2S;
            if (explicit_dir) {
                dir = a.fixed_dir;
            } else if (a.dirbits) {  // check_cache (src/common/cache.c:321-354), byte loaded with the span
                const uint64_t pktno = a.pkt_base + tile.first_pkt + lane;
                const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
                const uint32_t b = my_dirv ? my_dirb : 0u;
                dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
            }
#if TE_WK_EXP == 1  // diagnostics only: the skeleton without the edit (output = input)
            dir = TE_DIR_NOSEND;
#endif
            // tcprewrite.c:314-315: a record the cache says not to send is written unedited
            bool nosend = on && dir == TE_DIR_NOSEND && !explicit_dir;
            fl::State st;
            st.do_l4 = st.tail = false;
            st.dirty = 0;
            // phase A runs on every lane (it has no divergent branches); only lanes that edit
            // a packet keep its verdict and state
            const bool edit = on && !nosend && !fz_cut;
#if TE_WK_EXP == 2  // diagnostics only: window reads, no edit
            bool ok = true;
            {
                uint32_t x = 0;
#pragma unroll
                for (int i = 0; i < fl::NW; ++i) x ^= H[i];
                ok = x != 0x9e3779b9u;
                nosend = true;
            }
#else
            bool ok = MTU ? fl::phase_a<F>(H, caplen, len, part, dir, cfg, kn, a.v6_ok != 0, lut, st, mcut ? ecap : 0u)
                          : fl::phase_a<F>(H, ecap, elen, part, dir, cfg, kn, a.v6_ok != 0, lut, st, 0u, fz_recalc);
            if constexpr (VDEL) ok = ok && tagged;
            ok = ok || !(edit || fz_cut);  // (a cut record's plan assumed the shape too)
            // GROW / SHRINK: a record written unedited keeps its size; the scan placement takes it
            if constexpr (SZ != SZ_NONE) ok = ok && !nosend;
            st.tail = st.tail && edit;
#endif
            if (__ballot(!ok)) {  // a packet for the generic lane: it redoes this tile
                if (WIN) {  // (window mode: the exact path redoes the batch)
                    if (lane == 0) atomicOr(&a.w_flags[t], WIN_F_EDIT);
                } else if (lane == 0) {
                    a.tile_list[atomicAdd(a.list_cnt, 1u)] = t;
                }
                return false;
            }

            WK_STAMP(1)  // phase A
            // ---- chunk prefix for L4 bytes past the windows (large packets only) ----
            if (__ballot(st.tail)) {
                const uint32_t nch = (LDS_FRONT + g0 + tile.span_len + 15) >> 4;  // <= 64 * WK_KL
                uint32_t loc[WK_KL], tot = 0;
#pragma unroll
                for (int q = 0; q < WK_KL; ++q) {  // lane owns chunks [lane * KL, lane * KL + KL)
                    const uint32_t c = (uint32_t)lane * WK_KL + q;
                    uint32_t s = 0;
                    if (c < nch) {
                        const uint4 v = *(const uint4 *)(S + 16 * c);
                        s = fl::wsum(v.x) + fl::wsum(v.y) + fl::wsum(v.z) + fl::wsum(v.w);
                    }
                    loc[q] = tot;
                    tot += s;
                }
                const uint32_t incl = wave_scan_add(tot);
                const uint32_t base = incl - tot;
#pragma unroll
                for (int q = 0; q < WK_KL; ++q) {
                    const uint32_t c = (uint32_t)lane * WK_KL + q;
                    if (c < nch) P[c] = base + loc[q];
                }
                if (lane == 63) P[nch] = incl;
            }
            WK_LANES_SYNC();  // other lanes read the prefix

            WK_STAMP(2)  // chunk prefix
            // LDS dwords any lane writes back, as one wave-uniform mask: the per-dword tests
            // below are scalar branches.  A lane that did not change such a dword rewrites
            // it with its own packet's bytes (never past caplen), which is harmless.
            uint32_t todo = 0;
            if (edit) {
                todo = st.dirty;
                // VLAN pop: packet' dword i >= 4 is input dword i + 1; input dword 4 (the popped
                // TCI and the inner type field, unchanged) is never dirty
                if constexpr (VDEL) todo = (todo & 0xfu) | ((todo >> 4) << 5);
                todo |= (wa & 3u) ? (todo << 1) : 0u;
            }
            todo = wave_or(todo);
            // every written dword ends by packet offset 78 <= caplen + 16: no per-dword test
            const bool wide = !__ballot(edit && ecap < (uint32_t)fl::WEND - 16);
            // ---- phase B + write-back of the dwords phase A touched ----
            if (on) {
                if (edit) {
                    uint32_t tail = 0;
                    if (st.tail) {
                        const uint32_t pv = p + (VDEL ? 4u : 0u);  // packet' byte x is LDS byte pv + x
                        tail = lds_range_sum(S, P, pv + fl::WEND, pv + st.end);
                        if (p & 1) tail = fl::swap16(tail);  // absolute -> packet-relative pairing
                    }
                    fl::phase_b(H, st, tail);
                    // A dword is written whole when it ends within 16 bytes past caplen: past
                    // caplen lie the next record's pcap header bytes, which no lane edits before
                    // conv_hdr (after this loop), so their original bytes go back unchanged.  A
                    // dword further out would overlap the next record's packet bytes, which its
                    // own lane may be rewriting in this same loop.  (--efcs: past the new caplen
                    // lie the FCS bytes, written back unchanged; the store drops them.)
                    const uint32_t A = wa & ~3u, sh = wa & 3u;
#pragma unroll
                    for (int j = 0; j < fl::NW + XW; ++j) {
                        if (!((todo >> j) & 1u)) continue;
                        // input dword j: packet' dword j - (j >= 4) under the pop (dword 4 carries
                        // packet' dword 3's high half, the inner type, where the input has it)
                        const int hj = VDEL && j >= 4 ? j - 1 : j, hp = VDEL && j >= 5 ? j - 2 : j - 1;
                        const uint32_t cur = H[hj];
                        const uint32_t prev = j ? H[hp] : (d0 << (8 * (4 - sh)));
                        const uint32_t v = sh ? __builtin_amdgcn_alignbyte(cur, prev, 4 - sh) : cur;
                        if (wide || A + 4 * j + 4 <= p + caplen + 16) *(uint32_t *)(S + A + 4 * j) = v;
                    }
                }
                if (conv) conv_hdr(S + r0, swp, nsec);
                // after the write-back, which rewrote len's bytes
                if constexpr (GROW) hdr_add4(S, r0, 4u);
                if constexpr (SHRINK) hdr_add4(S, r0, (uint32_t)-4);
                if constexpr (MTU) {
                    if (mcut) hdr_put(S, r0, ecap);
                }
                if constexpr (FUZZ) {
                    if (fz_cut && fz_nl) hdr_put(S, r0, fz_nl);
                }
                // (window mode: no record numbers; every record it finishes is status 0, which
                // the caller writes for the whole batch)
                const uint8_t stb = nosend   ? (uint8_t)TE_ST_NOSEND
                                    : fz_cut ? (uint8_t)(TE_ST_RC_SOFT | (fz_nl ? 0 : TE_ST_ZEROCAP))
                                             : (uint8_t)0;
                if (!WIN) ((g_u8 *)a.status)[tile.first_pkt + lane] = stb;
            }
            if (conv && lane == (int)(npkt & 63u)) conv_hdr(S + LDS_FRONT + g0 + tile.span_len, swp, nsec);
            if (GROW && lane == (int)(npkt & 63u)) hdr_add4(S, LDS_FRONT + g0 + tile.span_len, 4u);
            if (SHRINK && lane == (int)(npkt & 63u)) hdr_add4(S, LDS_FRONT + g0 + tile.span_len, (uint32_t)-4);

            WK_LANES_SYNC();  // the store reads what every lane wrote back
            WK_STAMP(3)  // phase B
            // ---- store: the chunks that start in the span, then the leading bytes ----
            bool filled = false;
            if constexpr (GROW) {
                // record j's tag at output offset rel_j + 28 + 4 j (its input byte rel_j + 28 on)
                filled = wk_store_sized<true, TB>(S, P, gout, G0 + 4ull * tile.first_pkt, tile.span_len, npkt, g0,
                                                  my_rel + 28u + 4u * (uint32_t)lane, on, a.vlan_tag_word, lane,
                                                  stream && WK_SIZED_STREAM, pre_store);
            } else if constexpr (SHRINK) {
                const uint32_t Dj = my_rel + (VDEL ? 28u : 16u + ecap);
                filled = wk_store_sized<false, TB>(S, P, gout, G0 - 4ull * tile.first_pkt, tile.span_len, npkt, g0,
                                                   Dj - 4u * (uint32_t)lane, on, 0u, lane, stream && WK_SIZED_STREAM,
                                                   pre_store);
            } else if constexpr (MTU || FUZZ) {
                // the kept sizes -> output offsets; the tile's output at input offset - tcut[t]
                // (FUZZ: a dropped record keeps nothing, not even its header)
                const uint32_t osz = !on ? 0u : !FUZZ ? 16u + ecap : !fz_cut ? 16u + caplen : fz_nl ? 16u + fz_nl : 0u;
                const uint32_t incl = wave_scan_add(osz);
                const uint32_t out_len = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                const long long k0 = a.tcut[t], k1 = a.tcut[t + 1];
                const uint32_t cut = tile.span_len - out_len;
                if (lane == 0 && (long long)cut != k1 - k0) atomicOr(a.grow_bad, 1u);  // (a stale prediction)
                c_cut += cut;
                filled = wk_store_mtu<WK_KL + 1, FUZZ, MTU_NE>(S, LDS_FRONT + g0, P, gout, (uint64_t)((long long)G0 - k0),
                                                           out_len, npkt, my_rel, incl - osz, osz != 0u, lane,
                                                           stream && WK_MTU_STREAM, pre_store);
                if constexpr (FUZZ) {
                    c_drop += (unsigned long long)__popcll(__ballot(on && fz_cut && fz_nl == 0u));
                    c_soft += (unsigned long long)__popcll(__ballot(on && fz_cut));
                }
            } else {
                const uint64_t C0 = (G0 + 15) & ~15ull;
                const uint32_t nown = (uint32_t)((((E + 15) & ~15ull) - C0) >> 4);  // >= 1 (a 16-byte header)
                const uint8_t *src = S + LDS_FRONT + (uint32_t)(C0 - A0);
                // named registers, all reads in flight before the first store (left to itself the
                // scheduler reuses one register quad and waits out each read's LDS latency in turn)
                uint4 w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15;
#define WK_RD(k) \
        if constexpr (k < WK_KL) w##k = *(const uint4 *)(src + (umin32((uint32_t)lane + 64u * k, nown - 1u) << 4));
#define WK_WR(k)                                                                                       \
        if constexpr (k < WK_KL) {                                                                         \
            g_u4 *dk = (g_u4 *)(gout + C0 + ((uint64_t)umin32((uint32_t)lane + 64u * k, nown - 1u) << 4)); \
            if (stream && WK_PLAIN_STREAM)                                                                 \
                __builtin_nontemporal_store((u32x4){w##k.x, w##k.y, w##k.z, w##k.w}, (g_v4 *)dk);         \
            else                                                                                           \
                *dk = w##k;                                                                                \
        }
                WK_EACH(WK_RD)
                const uint32_t nlead = (uint32_t)(C0 - G0);
                const uint64_t q = (uint32_t)lane < nlead ? G0 + (uint32_t)lane : C0;  // others repeat byte C0
                const uint8_t lead = S[LDS_FRONT + (uint32_t)(q - A0)];
                // (the instances that read the cfg keep the fill after the stores: their
                //  registers spill with the span and the store data live together)
                if constexpr (TE_WK_FILL_EARLY && !WkCfg<F>::reads) {
                    WK_LANES_SYNC();  // (the image's reads before the next span's writes)
                    filled = pre_store();
                }
#if TE_WK_STORE_BARRIER
                __builtin_amdgcn_sched_barrier(0);
#endif
                WK_EACH(WK_WR)  // lanes past the span repeat its last chunk (same bytes)
#undef WK_RD
#undef WK_WR
                gout[q] = lead;
            }
#if TE_WK_STAMPS
            ++ntl;
#endif
            const uint32_t n_noedit = (uint32_t)__popcll(__ballot(on && !edit));
            c_pkts += npkt;
            c_bytes += tile.span_len;
            c_edited += npkt - n_noedit;
            return filled;
    };
    // one tile with DEPTH spans in flight.  Rf holds tile t's descriptor and per-lane
    // values (its chunks are in LDS already) and is reloaded with tile t + DEPTH * W;
    // Rn (DEPTH 2: tile t + W, in flight; DEPTH 1: Rf itself) goes to LDS after the store.
    te_tile_t dpre;  // descriptor of the next tile to issue
    auto step = [&](const uint32_t t, Span &Rf, Span &Rn) __attribute__((always_inline)) {
#if TE_WK_LANE_OPAQUE
        // lane-derived addresses are recomputed per tile instead of being hoisted out of
        // the loop and kept (or spilled) across it
        asm volatile("" : "+v"(lane));
#endif
        const te_tile_t tile = Rf.tl;
        const uint32_t my_rel = Rf.rel, my_dirb = Rf.dirb, my_fzs = Rf.fzs;
        const bool my_dirv = Rf.dirv;
        if (t + DEPTH * W < n_tiles) issue(Rf, dpre);  // in flight while this tile is edited and stored
        if (t + (DEPTH + 1) * W < n_tiles) dpre = tiles[t + (DEPTH + 1) * W];
        WK_STAMP(0)  // loop top + loads issued
        const bool filled = edit(t, tile, my_rel, my_dirb, my_dirv, my_fzs, [&]() __attribute__((always_inline)) {
            if (t + W < n_tiles) fill(Rn);
            return true;
        });
        WK_STAMP(4)  // stores issued
        if (!filled && t + W < n_tiles) fill(Rn);
        WK_LANES_SYNC();  // the next tile's lanes read what every lane filled
        WK_STAMP(5)  // next span -> LDS (waits for its loads)
    };

    if constexpr (WIN) {
        // ---- window mode: wave w takes windows w, w + W, ... ----
        if (blockIdx.x == 0 && threadIdx.x == 0) {  // te_win_check, next on the stream, writes them
            *a.win_bad = 0u;
            *a.win_tot = 0ull;
        }
        IdxArgs ia;
        ia.img = a.in;
        ia.len = a.win_len;
        ia.entry = a.win_entry;
        ia.entry_ptr = a.win_entry_ptr;
        ia.entry_sub = a.win_entry_sub;
        ia.base = a.win_base;
        ia.limit = a.win_limit;
        ia.sw = 0;
        ia.nsec = 0;
        uint8_t *const IMG = SB[wid];       // the staged window at IMG + LDS_FRONT
        uint16_t *const REL = RELB[WIN ? wid : 0];
        // TE_WIN_PREFETCH: the next window's staging in flight in registers while this one
        // is edited (A/B: on C2 it cost more in registers -- spills at 4 blocks/CU, or a
        // quarter of the occupancy at 3 -- than the overlap won)
        tew::Staging<WIN_S, WIN_OL, WIN_PRE> stg;
        if (TE_WIN_PREFETCH && w0 < a.nwin) tew::stage_load(ia, w0, stg);
        for (uint32_t k = w0; k < a.nwin; k += W) {
            if (!TE_WIN_PREFETCH) tew::stage_load(ia, k, stg);
            tew::stage_store(ia, k, stg, (uint32_t *)(IMG + LDS_FRONT));
#if TE_WK_STAMPS
            WK_STAMP(5)  // (window mode: the staging)
            const tew::Found fw =
                tew::find_window<WIN_S, WIN_OL, WIN_PRE, true, uint16_t>(ia, (uint32_t *)(IMG + LDS_FRONT), REL, k, fph);
            last_ = __builtin_amdgcn_s_memtime();
#else
            const tew::Found fw =
                tew::find_window<WIN_S, WIN_OL, WIN_PRE, true, uint16_t>(ia, (uint32_t *)(IMG + LDS_FRONT), REL, k);
#endif
            if (TE_WIN_PREFETCH && k + W < a.nwin) tew::stage_load(ia, k + W, stg);
            WK_STAMP(0)  // (window mode: the record discovery)
            const uint32_t wfl = fw.wstop | (fw.anytrim ? (uint32_t)IDX_TRIM : 0u);
            if (lane == 0) {
                a.w_entry[k] = fw.went;
                a.w_exit[k] = fw.wexit;
                a.w_flags[k] = wfl;
            }
            // a chain end or an empty record: te_win_check sends the batch to the exact path
            if (wfl || fw.nrec == 0) continue;
            // the bytes the window's last record reaches past the staged window, and the next
            // record's header (the last output chunk's bytes): loaded now, or (too long) left
            // to the exact path
            const uint64_t need = fw.wexit + 16;
            if (need > fw.staged_end) {
                if (need - fw.A0 > (uint64_t)(WIN_W + 48 + WIN_TAIL)) {
                    if (lane == 0) atomicOr(&a.w_flags[k], WIN_F_EDIT);
                    continue;
                }
                const uint64_t c0 = (fw.staged_end & ~15ull) - fw.A0, c1 = ((need + 15) & ~15ull) - fw.A0;
                for (uint64_t c = c0 + 16ull * (uint32_t)lane; c < c1; c += 1024)
                    *(uint4 *)(IMG + LDS_FRONT + c) = *(g_cu4 *)(gin + fw.A0 + c);
                WK_LANES_SYNC();
            }
            WK_STAMP(5)  // (window mode: the tail load, with the staging)
            // the tile cut walk_range makes: <= 64 records whose span fits the budget, a
            // record too large for it alone (then left to the exact path by edit())
            for (uint32_t s0 = 0; s0 < fw.nrec;) {
                const uint32_t i = s0 + (uint32_t)lane;
                const bool v = i < fw.nrec;
                const uint32_t r = v ? REL[i] : 0u, r1 = v ? REL[i + 1] : 0u;
                const uint32_t rs = REL[s0];
                const uint64_t t0 = fw.ws + rs;
                const bool fits = v && TE_CONTIG_FITS_IN((uint32_t)(t0 & 15), r1 - rs, (uint32_t)TB);
                const unsigned long long brk = __ballot(lane > 0 && (!v || !fits));
                const uint32_t len = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
                te_tile_t tl;
                tl.span_off = t0;
                tl.scratch_off = TE_NO_SCRATCH;
                tl.first_pkt = 0;
                tl.npkt = len;
                tl.span_len = REL[s0 + len] - rs;
                tl.flags = 0;
                const uint32_t my_rel = (uint32_t)lane < len ? r - rs : REL[s0 + len - 1] - rs;
                // the tile's image: its span start at S + LDS_FRONT + (span_off & 15)
                S = IMG + (uint32_t)((t0 & ~15ull) - fw.A0);
                WK_LANES_SYNC();
                edit(k, tl, my_rel, 0u, false, 0u, []() { return false; });
                WK_LANES_SYNC();
                WK_STAMP(4)  // (window mode: the edit's stores)
                s0 += len;
            }
        }
    } else {
    Span RA, RB;
    if (w0 < n_tiles) issue(RA, tiles[w0]);
    if (DEPTH == 2 && w0 + W < n_tiles) issue(RB, tiles[w0 + W]);
    if (w0 < n_tiles) fill(RA);
    if (w0 + DEPTH * W < n_tiles) dpre = tiles[w0 + DEPTH * W];
    if constexpr (DEPTH == 1) {
        for (uint32_t t = w0; t < n_tiles; t += W) step(t, RA, RA);
    } else {
        for (uint32_t t = w0; t < n_tiles; t += 2 * W) {
            step(t, RA, RB);
            if (t + W >= n_tiles) break;
            step(t + W, RB, RA);
        }
    }
    }
#undef WK_EACH
#if TE_WK_STAMPS
    if (lane == 0 && wid == 0 && (blockIdx.x % 128) == 0)
        printf("wstamps block %u tiles %llu: top %llu phaseA %llu prefix %llu phaseB %llu store %llu fill %llu\n",
               blockIdx.x, ntl, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5]);
    if constexpr (WIN) {
        if (lane == 0 && wid == 0 && (blockIdx.x % 128) == 0)
            printf("fstamps block %u: cand %llu walk %llu confirm %llu jacobi %llu positions %llu\n", blockIdx.x,
                   fph[0], fph[1], fph[2], fph[3], fph[4]);
    }
#endif
    if (lane == 0) {
        red[wid][0] = c_pkts;
        red[wid][1] = c_bytes;
        red[wid][2] = c_edited;
        red[wid][3] = c_cut;
        red[wid][4] = c_drop;
        red[wid][5] = c_soft;
    }
    __syncthreads();
    if (tid < TE_WK_SLOT_WORDS) {  // this block's totals (the host adds them up)
        unsigned long long s = 0;
        if (tid < 6) {
#pragma unroll
            for (int w = 0; w < WK_NW; ++w) s += red[w][tid];
        }
        a.slots[TE_WK_SLOT_WORDS * blockIdx.x + tid] = s;
    }
}

// ---------------------------------------------------------------------------
// te_win_check: the window mode's cross-window chain check, one thread a window: a window's
// first record must be where the chain left the nearest earlier window a record starts in
// (the first window's, the known first record), and a window without one must be passed
// over whole; a chain end, an empty record or a miss sends the batch to the exact path.
// The chain's end (the next pipeline chunk's first record) is the largest exit.
// ---------------------------------------------------------------------------
// The window-mode pipeline's per-chunk steps ride in the same launch (WinTail): one block
// adds the chunk's block totals and the edit's verdict bits to the call's accumulator
// {packets, bytes, edited, verdict} (the check blocks OR their own verdict in too), and
// WIN_HEAD_BLOCKS blocks copy the bytes before the chunk's first record -- the previous
// chunk's last record, edited there -- from the previous chunk's output image, so the
// chunk's output image holds its whole file range.
struct WinTail {
    unsigned long long *acc;  // null: a batch, no accumulator
    const unsigned long long *slots;
    uint32_t nslots, ncheck;   // the edit's blocks; the check's blocks
    const uint8_t *prev_out;   // null: no head copy (the first chunk, a batch)
    uint8_t *out;
    uint64_t head_max;         // a first record further in is no chain's: nothing copied
    uint64_t org;              // the image offset of the chunk's first file byte
};
constexpr uint32_t WIN_HEAD_BLOCKS = 64;

__device__ void win_head_copy(const FastArgs &a, const WinTail &w, uint32_t blk) {
    const uint64_t sub = a.win_entry_sub, org = w.org;
    // this chunk's first record (image offset): where the previous chunk's chain ended (a
    // chunk whose chain broke leaves no such position: the call's verdict sends the capture
    // to the exact path, and nothing is copied here)
    const uint64_t e = *(const volatile uint64_t *)a.win_entry_ptr - sub;
    if (e < org || e > w.head_max) return;
    const uint64_t t = blk * 256ull + threadIdx.x, nt = WIN_HEAD_BLOCKS * 256ull;
    if ((sub | org) & 15) {  // (not 16-byte pieces on both sides: byte by byte)
        for (uint64_t x = org + t; x < e; x += nt) w.out[x] = w.prev_out[x + sub];
        return;
    }
    // bytes [org, e) of this image are the previous image's [org + sub, e + sub)
    const uint64_t c1 = e & ~15ull;
    for (uint64_t c = org + 16 * t; c < c1; c += 16 * nt)
        *(uint4 *)(w.out + c) = *(const uint4 *)(w.prev_out + c + sub);
    if (t < 16 && c1 >= org && c1 + t < e) w.out[c1 + t] = w.prev_out[c1 + sub + t];
}

__global__ __launch_bounds__(256) void te_win_check(FastArgs a, unsigned long long *tot, WinTail w) {
    if (blockIdx.x >= w.ncheck) {
        const uint32_t b = blockIdx.x - w.ncheck;
        if (w.acc && b == 0) {  // the chunk's totals and the edit's verdict bits
            unsigned long long p = 0, by = 0, e = 0;
            for (uint32_t i = threadIdx.x; i < w.nslots; i += 256) {
                p += w.slots[TE_WK_SLOT_WORDS * i];
                by += w.slots[TE_WK_SLOT_WORDS * i + 1];
                e += w.slots[TE_WK_SLOT_WORDS * i + 2];
            }
            if (p) atomicAdd(&w.acc[0], p);
            if (by) atomicAdd(&w.acc[1], by);
            if (e) atomicAdd(&w.acc[2], e);

        } else if (w.prev_out) {
            win_head_copy(a, w, b - (w.acc ? 1u : 0u));
        }
        return;
    }
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    unsigned long long ex = 0;  // this window's exit (its last record's end), for the chain's end
    if (k < a.nwin) {
        // every load this window's check may need, issued together (the usual path reads
        // its own entry, exit and flags and the previous window's entry and exit; one
        // dependent walk back only past windows without a record)
        const uint64_t went = a.w_entry[k], wexit = a.w_exit[k];
        const uint32_t wf = a.w_flags[k];
        const uint64_t pent = k ? a.w_entry[k - 1] : IDX_NONE, pexit = k ? a.w_exit[k - 1] : 0ull;
        const uint64_t entry = a.win_entry_ptr ? *(const volatile uint64_t *)a.win_entry_ptr - a.win_entry_sub
                                               : a.win_entry;
        const uint32_t kE = (uint32_t)((entry - a.win_base) / WIN_WN);
        if (k >= kE) {
            bool bad = (wf & ~WIN_F_EDIT) != 0;
            if (wf & WIN_F_EDIT) {  // a record left to the exact path
                atomicOr(a.win_bad, 2u);
                if (w.acc) atomicOr(&w.acc[3], 2ull);
            }
            if (k == kE) {
                bad |= went != entry;
            } else {
                uint32_t j = k - 1, steps = 0;
                uint64_t ej = pent, xj = pexit;
                if (ej == IDX_NONE && j > kE) {  // (rare: windows without a record before this one)
                    while (j > kE && a.w_entry[j] == IDX_NONE && ++steps < 4096) --j;
                    ej = a.w_entry[j];
                    xj = a.w_exit[j];
                }
                if (ej == IDX_NONE) {
                    bad = true;
                } else if (went != IDX_NONE) {
                    bad |= xj != went;
                } else {
                    const uint64_t qe = a.win_base + (uint64_t)(k + 1) * WIN_WN;
                    bad |= xj < (qe < a.win_limit ? qe : a.win_limit);
                }
            }
            if (bad) {
                atomicOr(a.win_bad, 1u);
                if (w.acc) atomicOr(&w.acc[3], 1ull);
            }
            if (went != IDX_NONE) ex = wexit;
        }
    }
    // the chain's end: one atomic a wave on its windows' largest exit (one a window put
    // ~16K atomics on one address for C2's 1M records)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)ex, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(ex >> 32), o);
        const unsigned long long v = (unsigned long long)hi << 32 | lo;
        ex = v > ex ? v : ex;
    }
    if ((threadIdx.x & 63) == 0 && ex) atomicMax(&tot[0], ex);
}

// ===========================================================================
// te_q8_replay: the reference's static packet buffer, emulated (SURVEY Appendix B
// Q8).  tcprewrite memcpy's every record into one MAXPACKET buffer that is never
// cleared (tcprewrite.c:267-301), so an edit that reads past a record's captured
// bytes -- an IPv6 checksum over an overstated payload length, a TCP sequence field
// or an ARP address past caplen, remap_ipv6's stray write -- sees what earlier
// records left there.  The edit kernel lists each such written record with the
// buffer extent it read ([0, need)); one thread per listed record then rebuilds the
// buffer sequentially:
//   * walking back from the record, it finds the latest records whose memcpy
//     covers [0, need) (each older one only matters where it reached further), or
//     the capture's start, where the buffer is all zeros (safe_malloc, utils.c:38-48;
//     tcpedit_packet: the caller's own buffer).  The walk may go on into the records
//     just before the batch when the host staged them (the previous pipeline chunk's or
//     shard's last records, record numbers -npre .. -1);
//   * it replays tcpedit_packet over the emulated buffer for every record from there
//     on, in order, normalising each edit to the reference's in-place layout (the
//     encoders' memmove: the packet starts at the buffer start, bytes past its
//     extent keep their earlier values);
//   * the listed record's bytes then replace what the edit kernel wrote.
// A replay that itself meets bytes nobody has written yet (valid prefix V) or whose
// chain leaves this batch (a later pipeline chunk, a shard) fails and is counted in
// TE_CNT_Q8_FAILED; the host then reports the record instead of writing a guess.
// ===========================================================================
constexpr uint32_t Q8_HEAD = 512;                        // room for the record header's moves
constexpr uint32_t Q8_BUF = MAXPACKET + 4096;            // the emulated buffer (+ edits past MAXPACKET)
constexpr uint64_t Q8_SLOT = ((uint64_t)Q8_HEAD + Q8_BUF + 255) & ~255ull;
constexpr uint32_t Q8_MAX_CHAIN = 1u << 18;              // records a replay may walk back over
constexpr int Q8_BLOCK = 64;

struct Q8Args {
    LaunchArgs a;
    uint8_t *scratch;       // Q8_SLOT bytes per thread
    uint32_t n_threads;
    uint32_t file_start;    // record 0 of the batch is the capture's first record
    const uint8_t *init_buf;  // the initial buffer (tcpedit_packet: the caller's), else zeros
    uint32_t init_len;
    const uint8_t *pre;       // the records before the batch (-npre .. -1), or none
    const uint64_t *pre_off;
    uint32_t npre;
    uint32_t pre_file_start;  // record -npre is the capture's first
};
constexpr int64_t Q8_START = -(1ll << 40);    // q8_chain: from the first record there is
constexpr int64_t Q8_TOOLONG = -(1ll << 41);  // q8_chain: walked back too far

__device__ __forceinline__ uint32_t q8_tile(const LaunchArgs &a, uint32_t j) {
    uint32_t lo = 0, hi = a.n_tiles - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (a.tiles[mid].first_pkt <= j) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint64_t q8_rec(const LaunchArgs &a, uint32_t j) {
    return a.tiles[q8_tile(a, j)].span_off + a.pkt_rel[j];
}

// record j of the replay's range: the batch's, or (j < 0) one staged before it
__device__ __forceinline__ const uint8_t *q8_recp(const Q8Args &q, int64_t j) {
    return j >= 0 ? q.a.in + q8_rec(q.a, (uint32_t)j) : q.pre + q.pre_off[j + (int64_t)q.npre];
}

// the oldest record of the newest ones whose memcpy's cover [0, need) before record
// `pos` (each older one only matters where it reached further); Q8_START: the first
// record there is (the batch's, or the first staged before it)
__device__ int64_t q8_chain(const Q8Args &q, int64_t pos, uint32_t need) {
    const bool swp = q.a.in_swapped != 0;
    uint32_t cov = 0;
    int64_t j0 = Q8_START;
    uint32_t steps = 0;
    for (int64_t j = pos - 1; j >= -(int64_t)q.npre; --j) {
        if (++steps > Q8_MAX_CHAIN) return Q8_TOOLONG;
        const uint8_t *rh = q8_recp(q, j);
        const uint32_t fc = ld_hdr32(rh + 8, swp), pl = ld_hdr32(rh + 12, swp);
        const uint32_t cl = pl < fc ? pl : fc;  // the bytes tcprewrite.c:301 copied (the trimmed caplen)
        if (cl > cov) {
            cov = cl;
            j0 = j;
            if (cov >= need) return j0;
        }
    }
    return Q8_START;
}

enum { Q8_OK = 0, Q8_FAIL = 1, Q8_DEEPER = 2 };
#if TE_Q8_DEBUG  // (diagnostics builds) why a replay gave up
#define Q8_DBG(r) printf("q8 fail %d: record %u start %lld npre %u file_start %u\n", (r), i, (long long)start, \
                         q.npre, q.npre ? q.pre_file_start : q.file_start)
#else
#define Q8_DBG(r)
#endif

// replay records j0..i over the emulated buffer (j0 < 0: from the batch start, whose
// buffer is zeros or the caller's); Q8_DEEPER: record *jd read bytes past what the
// replay has (*needd), so it has to start further back
template <bool FZ>
__device__ int q8_replay_from(const Q8Args &q, const te_dev_cfg_t &cfg, int64_t start, uint32_t i, uint64_t out_off,
                              uint8_t *slot, int64_t *jd, uint32_t *needd) {
    const LaunchArgs &a = q.a;
    const bool swp = a.in_swapped != 0;
    uint8_t *buf = slot + Q8_HEAD;
    uint32_t V = 0;  // bytes [0, V) of the emulated buffer are known
    int64_t j0 = start;
    if (start == Q8_START) {
        // the bytes come from before every record there is: the capture's start (zeros),
        // else they are not here
        if (!(q.npre ? q.pre_file_start : q.file_start)) { Q8_DBG(1); return Q8_FAIL; }
        j0 = -(int64_t)q.npre;
        if (q.init_buf) {
            for (uint32_t x = 0; x < q.init_len; ++x) buf[x] = q.init_buf[x];
            V = q.init_len;
        } else {
            for (uint32_t x = 0; x < MAXPACKET; x += 16) *(uint4 *)(buf + x) = make_uint4(0, 0, 0, 0);
            V = MAXPACKET;
        }
    }
    for (int64_t j = j0; j <= (int64_t)i; ++j) {
        const uint8_t *rec = q8_recp(q, j);
        const uint32_t ts_sec = ld_hdr32(rec, swp), ts_frac = ld_hdr32(rec + 4, swp) / (a.in_nsec ? 1000u : 1u);
        const uint32_t fcap = ld_hdr32(rec + 8, swp), len = ld_hdr32(rec + 12, swp);
        if (fcap > MAX_SNAPLEN) { Q8_DBG(2); return Q8_FAIL; }
        const uint32_t caplen = len < fcap ? len : fcap;  // safe_pcap_next's trim (utils.c:159-162)
        for (uint32_t x = 0; x < caplen; ++x) buf[x] = rec[16 + x];  // tcprewrite.c:301
        if (caplen > V) V = caplen;
        if (j < 0 && (a.l2carry || a.jscan || (FZ && a.fuzz_mode == TE_FUZZ_APPLY)))
            { Q8_DBG(3); return Q8_FAIL; }  // (a staged record's carried state is not at hand)
        const uint64_t pktno = a.pkt_base + (uint64_t)j;
        int dir = TE_DIR_C2S;
        const bool explicit_dir = a.fixed_dir >= 0;
        if (explicit_dir) {
            dir = a.fixed_dir;
        } else if (a.dirbits) {
            const uint64_t idx = pktno >> 2;
            const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
            const uint8_t b = idx < a.dirbits_len ? a.dirbits[idx] : 0;
            dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
        }
        if (dir == TE_DIR_NOSEND && !explicit_dir) continue;  // written unedited: the buffer holds its input
        uint8_t *hdr = buf - 16;
        st32(hdr, ts_sec);
        st32(hdr + 4, ts_frac);
        st32(hdr + 8, caplen);
        st32(hdr + 12, len);
        Pkt pk;
        pk.d = buf;
        pk.caplen = caplen;
        pk.len = len;
        pk.phys = V;
        pk.avail = Q8_BUF - 64;
        pk.unsupported = false;
        pk.need = 0;
        pk.ext = caplen;
        pk.strict = true;
        pk.room = Q8_HEAD - 16;
        pk.l2carry = a.l2carry ? (uint8_t)(a.l2carry[j] & 1u) : 0;
        if (a.l2carry && (a.l2carry[j] >> 63)) { Q8_DBG(6); return Q8_FAIL; }  // (a poisoned carry, q18_keys)
        jnpr_carry(a, (uint64_t)j, pk);
        bool warned = false;
        const uint32_t fzs = (FZ && a.fuzz_mode == TE_FUZZ_APPLY) ? a.fuzz_state[j] : 0u;
        const int rc = tcpedit_packet<FZ, true>(pk, cfg, a.portlut, dir, warned, a.fuzz_mode, fzs);
        if (pk.unsupported) {  // bytes nobody wrote yet in this replay (or slot headroom)
            if (pk.need == NEED_NEVER || pk.need > MAXPACKET) { Q8_DBG(4); return Q8_FAIL; }
            *jd = j;
            *needd = pk.need;
            return Q8_DEEPER;
        }
        if (j == (int64_t)i) {
            if (rc == RC_ERROR || rc == RC_SOFT) { Q8_DBG(5); return Q8_FAIL; }  // cannot change the pass-1 layout
            g_u8 *o = (g_u8 *)a.out + out_off;
            const uint32_t oc = (uint32_t)o[8] | ((uint32_t)o[9] << 8) | ((uint32_t)o[10] << 16) |
                                ((uint32_t)o[11] << 24);
            if (oc != pk.caplen) { Q8_DBG(6); return Q8_FAIL; }
            for (uint32_t x = 0; x < pk.caplen; ++x) o[16 + x] = pk.d[x];
            g_u8 *st = (g_u8 *)a.status + i;
            const uint8_t old = *st;
            uint8_t nst = (uint8_t)(old & ~(TE_ST_UNSUPPORTED | TE_ST_WARNED | TE_ST_RC_MASK));
            nst |= rc == RC_WARN ? TE_ST_RC_WARN : TE_ST_RC_OK;
            if (warned) nst |= TE_ST_WARNED;
            *st = nst;
            const int dw = (warned ? 1 : 0) - ((old & TE_ST_WARNED) ? 1 : 0);
            if (dw) atomicAdd(&a.counters[TE_CNT_WARN], (unsigned long long)(long long)dw);
            return Q8_OK;
        }
        // back to the reference's in-place layout: the packet starts at the buffer start
        // (strict_tail kept pk.d + x == buffer offset x for every known x)
        const int sft = (int)(pk.d - buf);
        const uint32_t M = pk.ext > pk.phys ? pk.ext : pk.phys;
        if (sft < 0)  // the packet grew: it sits below the buffer start
            for (uint32_t x = M; x-- > 0;) buf[x] = pk.d[x];
        else if (sft > 0)  // it shrank: it sits above the buffer start
            for (uint32_t x = 0; x < M; ++x) buf[x] = pk.d[x];
        if (M > V) V = M;
    }
    { Q8_DBG(7); return Q8_FAIL; }
}

template <bool FZ>
__device__ bool q8_replay_one(const Q8Args &q, const te_dev_cfg_t &cfg, uint4 ent, uint8_t *slot) {
    const uint32_t i = ent.x, need = ent.y;
    const uint64_t out_off = (uint64_t)ent.z | ((uint64_t)ent.w << 32);
    if (need == NEED_NEVER || need > MAXPACKET) return false;
    int64_t start = q8_chain(q, i, need);
    // an earlier record of the replay may read past what it has: start further back
    for (int iter = 0; iter < 64; ++iter) {
        if (start == Q8_TOOLONG) return false;
        int64_t jd = 0;
        uint32_t nd = 0;
        const int r = q8_replay_from<FZ>(q, cfg, start, i, out_off, slot, &jd, &nd);
        if (r == Q8_OK) return true;
        if (r == Q8_FAIL || start == Q8_START) return false;
        const int64_t s2 = q8_chain(q, jd, nd);
        if (s2 != Q8_START && s2 >= start) return false;  // no progress
        start = s2;
    }
    return false;
}

template <bool FZ>
__global__ void __launch_bounds__(Q8_BLOCK) te_q8_replay(Q8Args q) {
    const LaunchArgs &a = q.a;
    const unsigned long long listed = *(volatile unsigned long long *)&a.counters[TE_CNT_UNSUPPORTED];
    const uint32_t n = (uint32_t)(listed < a.q8_cap ? listed : a.q8_cap);
    const uint32_t g = blockIdx.x * Q8_BLOCK + threadIdx.x;
    if (g == 0 && listed > a.q8_cap) atomicAdd(&a.counters[TE_CNT_Q8_FAILED], listed - a.q8_cap);
    uint8_t *slot = q.scratch + (uint64_t)g * Q8_SLOT;
    for (uint32_t e = g; e < n; e += q.n_threads)
        if (!q8_replay_one<FZ>(q, *a.cfg, a.q8_list[e], slot)) atomicAdd(&a.counters[TE_CNT_Q8_FAILED], 1ull);
}

}  // namespace

// persistent grid = the blocks that are resident at once (CUs x occupancy)
static int cu_count() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return cus;
}

static int resident_blocks(int slot_layout) {
    static int cached[2] = {0, 0};
    int &c = cached[slot_layout ? 1 : 0];
    if (c) return c;
    int cus = cu_count(), per_cu = 0;
    if (!cus) return 256;
    hipError_t e = slot_layout
                       ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, te_edit_tiles<MODE_SLOT>, BLOCK, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, te_edit_tiles<MODE_CONTIG>, BLOCK, 0);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    c = cus * per_cu;
    return c;
}

// ===========================================================================
// --fuzz-seed RNG states.  The reference draws one tcpr_random() (three LCG steps,
// utils.c:436-458) from a run-wide state for every record that reaches the fuzz
// step, in record order (tcpedit.c:250-258, fuzzing.c:87).  After the reach pass
// (status[i] = 1 for such a record) record i's state is the run's state advanced
// by 3 x (reaching records before i): a count, an exclusive scan and an LCG jump.
// words[0] is the context's running state, words[1] this launch's starting state.
// ===========================================================================
constexpr int FZ_PER_THREAD = 4, FZ_BLOCK = 256, FZ_PER_BLOCK = FZ_PER_THREAD * FZ_BLOCK;

__device__ __forceinline__ uint32_t lcg_jump(uint32_t x, uint64_t k) {  // k steps of n*1103515245+12345
    uint32_t am = 1, ap = 0, cm = 1103515245u, cp = 12345u;
    while (k) {
        if (k & 1) {
            am *= cm;
            ap = ap * cm + cp;
        }
        cp = (cm + 1u) * cp;
        cm *= cm;
        k >>= 1;
    }
    return am * x + ap;
}

__device__ __forceinline__ uint32_t fz_flags(const uint8_t *st, uint32_t n, uint32_t i0, uint32_t f[FZ_PER_THREAD]) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < FZ_PER_THREAD; ++k) {
        f[k] = i0 + k < n ? (st[i0 + k] & 1u) : 0u;
        c += f[k];
    }
    return c;
}

__global__ void __launch_bounds__(FZ_BLOCK) te_fuzz_count(const uint8_t *st, uint32_t n, uint32_t *blk) {
    __shared__ uint32_t wsum[FZ_BLOCK / 64];
    uint32_t f[FZ_PER_THREAD], tot;
    const uint32_t c = fz_flags(st, n, blockIdx.x * FZ_PER_BLOCK + threadIdx.x * FZ_PER_THREAD, f);
    block_exscan<FZ_BLOCK>(c, wsum, tot);
    if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// one block: exclusive scan of the block counts in place, then the state words
// (words[2] = reaching records; advance = 0 leaves the running state alone, 2 takes the
// states' start from it and leaves it: the Q18 carry-out of a shard before its edit)
__global__ void __launch_bounds__(1024) te_fuzz_scan(uint32_t *blk, uint32_t nblk, uint32_t *words, int advance) {
    __shared__ uint32_t wsum[1024 / 64];
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblk; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nblk ? blk[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exscan<1024>(v, wsum, tot);
        if (i < nblk) blk[i] = (uint32_t)carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        const uint32_t s0 = words[0];
        words[2] = (uint32_t)carry;
        if (advance) words[1] = s0;
        if (advance == 1) words[0] = lcg_jump(s0, 3ull * carry);
    }
}

__global__ void __launch_bounds__(FZ_BLOCK) te_fuzz_states(const uint8_t *st, uint32_t n, const uint32_t *blk,
                                                           const uint32_t *words, uint32_t *states) {
    __shared__ uint32_t wsum[FZ_BLOCK / 64];
    uint32_t f[FZ_PER_THREAD], tot;
    const uint32_t i0 = blockIdx.x * FZ_PER_BLOCK + threadIdx.x * FZ_PER_THREAD;
    const uint32_t c = fz_flags(st, n, i0, f);
    const uint32_t rank = blk[blockIdx.x] + block_exscan<FZ_BLOCK>(c, wsum, tot);
    // one jump to the thread's first record, then one draw (three steps) per reaching record
    uint32_t x = lcg_jump(words[1], 3ull * rank);
#pragma unroll
    for (int k = 0; k < FZ_PER_THREAD; ++k) {
        if (i0 + k < n) states[i0 + k] = x;
        if (f[k]) x = ((x * 1103515245u + 12345u) * 1103515245u + 12345u) * 1103515245u + 12345u;
    }
}

extern "C" int te_fast_grid(void) {
    static int c = 0;
    if (c) return c;
    int cus = cu_count(), per_cu = 0;
    if (!cus) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, te_fast_tiles, FKB, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    c = cus * per_cu;
    return c;
}

// the te_wave_tiles instances built (TE_FF_* masks), smallest first: a launch takes
// the first whose mask covers the config's option groups
// TE_WK_DEPTH_LEAN=2 gives the lean instances two spans in flight per wave (their
// registers allow it at 4 waves per SIMD).  Measured on MI355X: C2 -0.6 %, C5 +2.5 %
// time, so one span is the default.
#ifndef TE_WK_DEPTH_LEAN
#define TE_WK_DEPTH_LEAN 1
#endif
#ifndef TE_WK_DEPTH_SMALL
#define TE_WK_DEPTH_SMALL 1
#endif
// (TE_FF_INCR is a mode, not an option group: an instance with it keeps the incremental
// checksums of a run without --fixcsum, so a launch takes one whose INCR bit matches)
#ifndef TE_WK_DEPTH_READS
#define TE_WK_DEPTH_READS 1
#endif
#define TE_FF_ALLH (TE_FF_ALL | TE_FF_HDR)
#define DR TE_WK_DEPTH_READS
#ifndef TE_WK_SIZED_LEAN
#define TE_WK_SIZED_LEAN 0
#endif
#if TE_WK_SIZED_LEAN
// (the static +-4 changes without an edit that reads the cfg, and C4's MACs + endpoints)
#define TE_WAVE_SIZED_LEAN(X)                                                                        \
    X(0u, 1, SZ_GROW) X(0u, 1, SZ_VDEL) X(0u, 1, SZ_EFCS) X(TE_FF_MAC | TE_FF_RWIP, 1, SZ_GROW)
#else
#define TE_WAVE_SIZED_LEAN(X)
#endif
#define TE_WAVE_INSTANCES(X)                                                                         \
    X(0u, TE_WK_DEPTH_LEAN, SZ_NONE) X(TE_FF_SEED, TE_WK_DEPTH_LEAN, SZ_NONE)                          \
    X(TE_FF_SMALL, TE_WK_DEPTH_SMALL, SZ_NONE) X(TE_FF_SEED | TE_FF_SMALL, TE_WK_DEPTH_SMALL, SZ_NONE)  \
    X(TE_FF_SEED | TE_FF_INCR | TE_FF_SMALL, TE_WK_DEPTH_SMALL, SZ_NONE)                               \
    X(TE_FF_PORTMAP | TE_FF_RWIP, DR, SZ_NONE) X(TE_FF_ALL, DR, SZ_NONE) X(TE_FF_ALLH, DR, SZ_NONE)    \
    X(TE_FF_SEED | TE_FF_INCR, TE_WK_DEPTH_LEAN, SZ_NONE) X(TE_FF_HDR | TE_FF_INCR, DR, SZ_NONE)        \
    X(TE_FF_ALLX, DR, SZ_NONE)                                                                        \
    X(TE_FF_PORTMAP | TE_FF_RWIP | TE_FF_SMALL, 1, SZ_NONE) X(TE_FF_ALL | TE_FF_SMALL, 1, SZ_NONE)      \
    X(TE_FF_ALLH | TE_FF_SMALL, 1, SZ_NONE) X(TE_FF_HDR | TE_FF_INCR | TE_FF_SMALL, 1, SZ_NONE)         \
    X(TE_FF_ALLX | TE_FF_SMALL, 1, SZ_NONE)                                                           \
    TE_WAVE_SIZED_LEAN(X)                                                                             \
    X(TE_FF_ALL, DR, SZ_GROW) X(TE_FF_ALLH, DR, SZ_GROW) X(TE_FF_ALLX, DR, SZ_GROW)                   \
    X(TE_FF_ALLH, DR, SZ_VDEL) X(TE_FF_ALLX, DR, SZ_VDEL) X(TE_FF_ALLH, DR, SZ_EFCS) X(TE_FF_ALLX, DR, SZ_EFCS)  \
    X(0u, 1, SZ_MTU) X(TE_FF_ALLH, 1, SZ_MTU)                                                          \
    X(TE_FF_INCR, 1, SZ_FUZZ) X(0u, 1, SZ_FUZZ) X(TE_FF_RWIP | TE_FF_INCR, 1, SZ_FUZZ)                  \
    X(TE_FF_RWIP, 1, SZ_FUZZ)
#define TE_WIN_INSTANCES(X)                                                                           \
    X(0u, 1, SZ_NONE) X(TE_FF_SEED, 1, SZ_NONE) X(TE_FF_PORTMAP | TE_FF_RWIP, 1, SZ_NONE)             \
    X(TE_FF_ALL, 1, SZ_NONE) X(TE_FF_ALLH, 1, SZ_NONE) X(TE_FF_SEED | TE_FF_INCR, 1, SZ_NONE)          \
    X(TE_FF_HDR | TE_FF_INCR, 1, SZ_NONE) X(TE_FF_ALLX, 1, SZ_NONE)
static struct {
    uint32_t feat;
    int sz;
    const void *fn;
    int grid;  // resident blocks of this instance (CUs x its occupancy), 0 until asked
} wave_inst[] = {
#define TE_WI(f, d, g) {f, g, (const void *)te_wave_tiles<f, d, g>, 0},
    TE_WAVE_INSTANCES(TE_WI)
#undef TE_WI
};

// window-mode instances: the size-preserving ones
static struct {
    uint32_t feat;
    const void *fn;
    int grid;
} win_inst[] = {
#define TE_WW(f, d, g) {f, (const void *)te_wave_tiles<f, d, g, true>, 0},
    TE_WIN_INSTANCES(TE_WW)
#undef TE_WW
};

static uint32_t fast_feat(const te_dev_cfg_t *c);
// the first (smallest) instance covering the config's option groups and size change;
// TCPEDIT_HIP_WAVE_FEAT=<mask> adds groups to the choice (A/B runs)
// (TE_FF_SMALL in `want`: the small-tile instance of the same groups if there is one, else the
//  other; the INCR and SMALL modes match exactly)
static int wave_pick(uint32_t want, int sz) {
    static const uint32_t feat_env =
        getenv("TCPEDIT_HIP_WAVE_FEAT") ? (uint32_t)atoi(getenv("TCPEDIT_HIP_WAVE_FEAT")) : 0u;
    want |= feat_env;
    if (sz == SZ_MTU) want &= ~TE_FF_INCR;  // (--mtu-trunc recomputes every IP packet's checksums)
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t w = pass ? want & ~TE_FF_SMALL : want;
        for (int k = 0; k < (int)(sizeof(wave_inst) / sizeof(wave_inst[0])); ++k)
            if (wave_inst[k].sz == sz && (w & ~wave_inst[k].feat) == 0 &&
                ((w ^ wave_inst[k].feat) & (TE_FF_INCR | TE_FF_SMALL)) == 0)
                return k;
        if (!(want & TE_FF_SMALL)) break;
    }
    return -1;
}

// (--seed sets rewrite_ip too, tcpedit parse_args.c:218-238, but rewrite_ipv4l3 /
// rewrite_ipv6l3 with no map change nothing and return 0, edit_packet.c:787-878: a seed-only
// config runs the lean SEED instance, not the cfg-reading address-map one)
static uint32_t fast_feat(const te_dev_cfg_t *c) {
    const bool maps = c->n_srcipmap || c->n_dstipmap || c->n_cidrmap1 || c->n_cidrmap2;
    return ((c->mac_mask || c->n_subs || c->random_set) ? TE_FF_MAC : 0u) | (c->has_portmap ? TE_FF_PORTMAP : 0u) |
           ((c->rewrite_ip && maps) ? TE_FF_RWIP : 0u) | (c->seed ? TE_FF_SEED : 0u) |
           ((c->tos >= 0 || c->ttl_mode != TE_TTL_OFF || c->tclass >= 0 || c->flowlabel >= 0 ||
             c->tcp_sequence_enable)
                ? TE_FF_HDR
                : 0u) |
           (c->fixcsum ? 0u : TE_FF_INCR);
}

// the wave lane's grid cut to the waves that give every wave the same number of tiles
// (ceil(tiles / resident waves) rounds), instead of all resident waves with a last round
// only some of them take: the same rounds, no lone tail (A/B: C5 0.631 -> 0.646, C2, C3,
// seed within 0.3 %; TCPEDIT_HIP_WAVE_BALANCE=0 launches every resident wave)
static bool wave_balance() {
    static int v = -1;
    if (v < 0) v = getenv("TCPEDIT_HIP_WAVE_BALANCE") ? atoi(getenv("TCPEDIT_HIP_WAVE_BALANCE")) != 0 : 1;
    return v != 0;
}

static int wave_inst_grid(int k) {
    if (wave_inst[k].grid) return wave_inst[k].grid;
    int cus = cu_count(), per_cu = 0;
    if (!cus) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wave_inst[k].fn, WKB, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    wave_inst[k].grid = cus * per_cu;
    return wave_inst[k].grid;
}

// the tile budget of the wave-lane instance a config launches (the host cuts tiles to it)
static int wave_pick(uint32_t want, int sz);
extern "C" uint32_t te_wave_tile_bytes(const te_dev_cfg_t *c, int sz, int small) {
    const int k = wave_pick(fast_feat(c) | (small ? TE_FF_SMALL : 0u), sz);
    if (k < 0) return TE_WK_TILE_BYTES;
    const bool reads = (wave_inst[k].feat & (TE_FF_MAC | TE_FF_PORTMAP | TE_FF_RWIP | TE_FF_HDR)) != 0;
    const int sz_ = wave_inst[k].sz;
    if ((sz_ == SZ_MTU || sz_ == SZ_FUZZ) && TE_WK_CUT_TILE_BYTES) return TE_WK_CUT_TILE_BYTES;
    if (sz_ == SZ_GROW || sz_ == SZ_VDEL || sz_ == SZ_EFCS) return reads ? TE_WK_SIZED_TILE_BYTES : TE_WK_SIZED_LEAN_TILE_BYTES;
    return reads ? (sz_ == SZ_NONE ? ((wave_inst[k].feat & TE_FF_SMALL) ? TE_WK_TILE_BYTES : TE_WK_READS_TILE_BYTES)
                                   : TE_WK_TILE_BYTES)
           : wave_inst[k].sz == SZ_NONE && !(wave_inst[k].feat & TE_FF_SMALL) ? TE_WK_BIG_TILE_BYTES
                                                                            : TE_WK_LEAN_TILE_BYTES;
}

// the waves a config's wave-lane launch runs (its instance's resident grid x 4): the host
// balances a small batch's tile cut to a whole number of rounds of them
extern "C" uint32_t te_wave_waves(const te_dev_cfg_t *c, int sz, int small) {
    const int k = wave_pick(fast_feat(c) | (small ? TE_FF_SMALL : 0u), sz);
    return k < 0 ? 0u : (uint32_t)wave_inst_grid(k) * (uint32_t)WK_NW;
}

// the largest wave-lane grid of any instance (the host sizes the per-block slots by it)
extern "C" int te_wave_grid(void) {
    static int c = 0;
    if (c) return c;
    int m = 0;
    for (int k = 0; k < (int)(sizeof(wave_inst) / sizeof(wave_inst[0])); ++k) {
        const int g = wave_inst_grid(k);
        m = g > m ? g : m;
    }
    c = m;
    return c;
}

// ---------------------------------------------------------------------------
// C-ABI launch wrapper (called from the C host code, no torch types)
// ---------------------------------------------------------------------------
static void fill_args(LaunchArgs &a, const te_launch_t *L) {
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
    a.rec0 = L->rec0;
    a.static_off = (uint32_t)L->static_off;
    a.static_grow = (uint32_t)L->static_grow;
    a.static_shrink = (uint32_t)L->static_shrink;
    a.grow_bad = L->grow_bad;
    a.tcut = (const long long *)L->tcut;
    a.static_mtu = (uint32_t)(L->static_mtu || L->static_fz);  // (placement by tcut)
    a.tile_list = nullptr;
    a.list_cnt = nullptr;
    a.counters_next = nullptr;
    a.fuzz_mode = TE_FUZZ_OFF;
    a.fuzz_state = nullptr;
    a.q8_list = (uint4 *)L->q8_list;
    a.q8_cap = L->q8_cap;
    a.l2carry = (const unsigned long long *)L->l2carry;
    a.q18_keys = nullptr;
    a.jscan = (const unsigned long long *)L->jscan;
    a.jstates = L->jstates;
    a.jctx = L->jctx;
}

// ===========================================================================
// a Linux cooked (SLL/SLL2) decoder into the en10mb encoder without
// --enet-dmac.  Every C2S record that reaches the encoder's address step sets the
// encoder's dst_modified (its first 6 bytes against the context's zero destination,
// en10mb.c:612-615); an S2C record leaves it, and the multicast MAC update of every
// record reads it (en10mb.c:868-882).  So a record sees the value of the last C2S record
// at or before it: one thread per record writes key[j + 1] = ((j + 1) << 1) | value for a
// C2S record (0 for the others), key[0] carries the context's value from the previous
// launch, and an inclusive max scan gives each record its predecessor's (scan[j]); the
// last entry goes back to the context word for the next launch.
// ===========================================================================
__global__ __launch_bounds__(256) void te_l2carry_mark(LaunchArgs a, unsigned long long *key, const uint32_t *word) {
    if (blockIdx.x == 0 && threadIdx.x == 0) key[0] = *word & 1u;
    const te_tile_t tile = a.tiles[blockIdx.x];
    if (threadIdx.x >= tile.npkt) return;
    const uint32_t j = tile.first_pkt + threadIdx.x;
    const te_dev_cfg_t &cfg = *a.cfg;
    const bool swp = a.in_swapped != 0;
    const uint8_t *rec = a.in + tile.span_off + a.pkt_rel[j];
    uint32_t caplen = ld_hdr32(rec + 8, swp);
    const uint32_t len = ld_hdr32(rec + 12, swp);
    if (len < caplen) caplen = len;                         // safe_pcap_next (utils.c:159-162)
    if (cfg.efcs && len > 4 && caplen == len) caplen -= 4;  // tcpedit.c:78-84
    int dir = TE_DIR_C2S;
    if (a.fixed_dir >= 0) {
        dir = a.fixed_dir;
    } else if (a.dirbits) {
        const uint64_t pktno = a.pkt_base + j;
        const uint64_t idx = pktno >> 2;
        const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
        const uint8_t b = idx < a.dirbits_len ? a.dirbits[idx] : 0;
        dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
    }
    // a writer: a C2S record that reaches the encoder's address step -- the decoder's proto
    // and decode succeed (tcpedit.c:96, dlt_plugins.c:210-238) and en10mb.c:544-585's length
    // checks pass -- run by the edit's own decoder functions over the record in HBM
    Pkt pk;
    pk.d = const_cast<uint8_t *>(rec + 16);
    pk.caplen = caplen;
    pk.len = len;
    pk.phys = pk.avail = pk.ext = caplen;
    pk.unsupported = false;
    pk.need = 0;
    pk.strict = false;
    // (a Juniper frame that is a TCPEDIT_WARN one decodes to the carried state, jnpr_carry)
    jnpr_carry(a, j, pk);
    Dec s;
    s.dst_modified = false;
    const bool decoded = dir != TE_DIR_NOSEND && decoder_proto(pk, cfg) >= 0 && foreign_decode(pk, cfg, s) != RC_ERROR;
    const int pktlen = (int)caplen;
    const bool writer = decoded && dir == TE_DIR_C2S && pktlen >= 14 && pktlen >= s.l2len &&
                        pktlen + 14 - s.l2len <= (int)MAXPACKET;
    // dst_modified: the frame's first 6 bytes (the encoder's memmove leaves them) against
    // the decoded destination (en10mb.c:612-615)
    bool nz = false;
    if (writer)
        for (int i = 0; i < 6; ++i) nz |= pk.d[i] != s.dstaddr[i];
    // the first whole Juniper inner decode makes the sub-decoder's extra the encoder's
    // (dlt_utils.c:261-263): the records after it read its dst_modified, false until a C2S
    // record writes it -- a writer of false unless it writes itself
    uint32_t hl = 0;
    const bool first = decoded && pk.jnone && cfg.decoder == TE_DEC_JNPR && jnpr_header(pk.d, caplen, hl) == RC_OK;
    key[j + 1] = writer ? ((unsigned long long)(j + 1) << 1 | (nz ? 1u : 0u))
                        : first ? (unsigned long long)(j + 1) << 1 : 0ull;
}

// ===========================================================================
// DLT_JUNIPER_ETHER into an encoder that reads the decoder state (en10mb, user, hdlc): a
// frame whose extensions are not Ethernet is a TCPEDIT_WARN (jnpr_ether.c:269-272) and is
// encoded with the state the last whole inner decode left in the context -- its addresses
// and proto (dlt_utils.c:249-271) and, by the extra pointer, the en10mb sub-decoder's VLAN
// fields.  te_jnpr_mark keys each record that decodes whole (the decoder's proto and
// decode succeed, tcpedit.c:96, dlt_plugins.c:210-238) with its position and stores its
// state; an inclusive max scan gives each record the last such record before it, and
// te_jnpr_save leaves the launch's last state in the context for the next launch.
// ===========================================================================
__global__ __launch_bounds__(256) void te_jnpr_mark(LaunchArgs a, unsigned long long *key, te_jstate_t *states) {
    if (blockIdx.x == 0 && threadIdx.x == 0) key[0] = 0;
    const te_tile_t tile = a.tiles[blockIdx.x];
    if (threadIdx.x >= tile.npkt) return;
    const uint32_t j = tile.first_pkt + threadIdx.x;
    const te_dev_cfg_t &cfg = *a.cfg;
    const bool swp = a.in_swapped != 0;
    const uint8_t *rec = a.in + tile.span_off + a.pkt_rel[j];
    uint32_t caplen = ld_hdr32(rec + 8, swp);
    const uint32_t len = ld_hdr32(rec + 12, swp);
    if (len < caplen) caplen = len;                         // safe_pcap_next (utils.c:159-162)
    if (cfg.efcs && len > 4 && caplen == len) caplen -= 4;  // tcpedit.c:78-84
    int dir = TE_DIR_C2S;
    if (a.fixed_dir >= 0) {
        dir = a.fixed_dir;
    } else if (a.dirbits) {
        const uint64_t pktno = a.pkt_base + j;
        const uint64_t idx = pktno >> 2;
        const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
        const uint8_t b = idx < a.dirbits_len ? a.dirbits[idx] : 0;
        dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
    }
    Pkt pk;
    pk.d = const_cast<uint8_t *>(rec + 16);
    pk.caplen = caplen;
    pk.len = len;
    pk.phys = pk.avail = pk.ext = caplen;
    pk.unsupported = false;
    pk.need = 0;
    pk.strict = false;
    uint32_t hl = 0;
    Dec s;
    s.dst_modified = false;
    const bool whole = dir != TE_DIR_NOSEND && decoder_proto(pk, cfg) >= 0 &&
                       jnpr_header(pk.d, caplen, hl) == RC_OK && foreign_decode(pk, cfg, s) == RC_OK;
    if (whole) {
        te_jstate_t st;
        for (int i = 0; i < 6; ++i) {
            st.dstaddr[i] = s.dstaddr[i];
            st.srcaddr[i] = s.srcaddr[i];
        }
        st.proto = (uint16_t)s.proto;
        st.vlan_tag = s.vlan_tag;
        st.vlan_pri = s.vlan_pri;
        st.vlan_cfi = s.vlan_cfi;
        st.vlan_proto = s.vlan_proto;
        st.pad0_ = 0;
        st.vlan_offset = s.vlan_offset;
        st.vlan = (uint8_t)s.vlan;
        st.pad1_[0] = st.pad1_[1] = st.pad1_[2] = 0;
        states[j + 1] = st;
    }
    key[j + 1] = whole ? (unsigned long long)(j + 1) : 0ull;
}

// the launch's last whole decode (if any) becomes the context's carried state
__global__ void te_jnpr_save(const unsigned long long *scan, const te_jstate_t *states, uint32_t n, te_jctx_t *ctx,
                             te_jctx_t *out) {
    if (threadIdx.x != 0) return;
    const unsigned long long i = scan[n];
    te_jctx_t c;
    if (out) {  // the launch's own: none unless it has a whole decode
        c.valid = TE_JC_NONE;
        for (int k = 0; k < 3; ++k) c.pad_[k] = 0;
        c.st = te_jstate_t{};
    } else {
        c = *ctx;
    }
    if (i) {
        c.st = states[i];
        c.valid = TE_JC_VALID;
    }
    if (out) *out = c;
    else *ctx = c;
}

__global__ void te_l2carry_save(const unsigned long long *scan, uint32_t n, uint32_t *word) {
    if (threadIdx.x == 0) *word = (uint32_t)(scan[n] & 1u);
}

struct MaxU64 {
    __device__ __forceinline__ unsigned long long operator()(unsigned long long x, unsigned long long y) const {
        return x > y ? x : y;
    }
};

extern "C" size_t te_l2carry_temp_bytes(uint32_t n_pkts) {
    size_t t = 0;
    if (hipcub::DeviceScan::InclusiveScan(nullptr, t, (const unsigned long long *)nullptr,
                                          (unsigned long long *)nullptr, MaxU64(), (int)n_pkts + 1) != hipSuccess)
        return 0;
    return t;
}

static void launch_generic(bool fz, bool anydec, bool slot, int grid, hipStream_t stream, const LaunchArgs &a);

// the keys and the scan before the edit (the edit then reads L->l2carry).  Under
// --fuzz-seed (a.fuzz_mode APPLY, the states drawn) a fuzzed record decodes and encodes a
// second time, so its last write is known only from its edit: a mark run of the edit
// writes the keys of the records it edits over te_l2carry_mark's (its output, counters and
// look-back words are the real run's to redo: `grid` blocks, then the zeroed region again)
static int l2carry_prepare(te_launch_t *L, const LaunchArgs &a, hipStream_t stream, int grid = 0) {
    if (!L->l2carry) return 0;
    if (!L->l2carry_keys || !L->l2carry_word || !L->l2carry_tmp || L->n_tiles == 0) return -1;
    hipLaunchKernelGGL(te_l2carry_mark, dim3(L->n_tiles), dim3(256), 0, stream, a,
                       (unsigned long long *)L->l2carry_keys, (const uint32_t *)L->l2carry_word);
    if (a.fuzz_mode == TE_FUZZ_APPLY) {
        if (grid < 1) return -1;
        LaunchArgs m = a;
        m.q18_keys = (unsigned long long *)L->l2carry_keys;
        m.l2carry = nullptr;
        m.q8_list = nullptr;
        launch_generic(true, L->any_dec != 0, L->slot_layout != 0, grid, stream, m);
        if (hipMemsetAsync(L->zero_region, 0, L->zero_bytes, stream) != hipSuccess) return -1;
    }
    size_t tb = L->l2carry_tmp_bytes;
    if (hipcub::DeviceScan::InclusiveScan(L->l2carry_tmp, tb, (const unsigned long long *)L->l2carry_keys,
                                          (unsigned long long *)L->l2carry, MaxU64(), (int)L->n_pkts + 1,
                                          stream) != hipSuccess)
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the Juniper state keys and scan before the edit (and before the fuzz reach pass: a
// warning frame's encode decides whether it reaches the fuzz step)
static int jnpr_prepare(te_launch_t *L, const LaunchArgs &a, hipStream_t stream) {
    if (!L->jscan) return 0;
    if (!L->jkeys || !L->jstates || !L->jctx || !L->jtmp || L->n_tiles == 0) return -1;
    hipLaunchKernelGGL(te_jnpr_mark, dim3(L->n_tiles), dim3(256), 0, stream, a, (unsigned long long *)L->jkeys,
                       L->jstates);
    size_t tb = L->jtmp_bytes;
    if (hipcub::DeviceScan::InclusiveScan(L->jtmp, tb, (const unsigned long long *)L->jkeys,
                                          (unsigned long long *)L->jscan, MaxU64(), (int)L->n_pkts + 1,
                                          stream) != hipSuccess)
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the keys and the scan alone (tcpedit_batch_l2carry_out: a shard's carry-out before any
// shard edits, so the ranks can exchange them); the Juniper state scan first (a warning
// frame's destination is the carried one)
extern "C" int te_launch_l2carry(te_launch_t *L, hipStream_t stream) {
    LaunchArgs a;
    fill_args(a, L);
    if (jnpr_prepare(L, a, stream) != 0) return -1;
    return l2carry_prepare(L, a, stream);
}

// the Juniper state scan alone and the state the launch would leave (a shard's carry-out:
// it does not depend on the carry-in, a whole decode reads none)
extern "C" int te_launch_jnpr(te_launch_t *L, te_jctx_t *out, hipStream_t stream) {
    LaunchArgs a;
    fill_args(a, L);
    if (!L->jscan || jnpr_prepare(L, a, stream) != 0) return -1;
    hipLaunchKernelGGL(te_jnpr_save, dim3(1), dim3(64), 0, stream, (const unsigned long long *)L->jscan, L->jstates,
                       L->n_pkts, L->jctx, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" uint64_t te_q8_slot_bytes(void) { return Q8_SLOT; }

// te_q8_replay over the records the last edit of this launch listed (the counter on the
// device says how many: a grid of q8_threads reads it and returns when it is 0)
extern "C" int te_launch_q8(te_launch_t *L, hipStream_t stream) {
    Q8Args q;
    fill_args(q.a, L);
    if (L->fuzz_states) {
        q.a.fuzz_mode = TE_FUZZ_APPLY;
        q.a.fuzz_state = L->fuzz_states;
    }
    q.scratch = (uint8_t *)L->q8_scratch;
    q.n_threads = L->q8_threads;
    q.file_start = (uint32_t)L->q8_file_start;
    q.init_buf = L->q8_init;
    q.init_len = L->q8_init_len;
    q.pre = L->q8_npre ? L->q8_pre : nullptr;
    q.pre_off = L->q8_npre ? L->q8_pre_off : nullptr;
    q.npre = L->q8_pre && L->q8_pre_off ? L->q8_npre : 0u;
    q.pre_file_start = (uint32_t)L->q8_pre_file_start;
    if (!q.scratch || q.n_threads == 0 || q.n_threads % Q8_BLOCK || !L->q8_list || L->n_tiles == 0) return -1;
    if (q.a.fuzz_mode == TE_FUZZ_APPLY)
        hipLaunchKernelGGL(te_q8_replay<true>, dim3(q.n_threads / Q8_BLOCK), dim3(Q8_BLOCK), 0, stream, q);
    else
        hipLaunchKernelGGL(te_q8_replay<false>, dim3(q.n_threads / Q8_BLOCK), dim3(Q8_BLOCK), 0, stream, q);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the generic lane's instance: fuzzing (FZ), the other decoders/encoders (AD), the layout
static void launch_generic(bool fz, bool ad, bool slot, int grid, hipStream_t stream, const LaunchArgs &a) {
#define TE_GL(M, F, D) hipLaunchKernelGGL((te_edit_tiles<M, F, D>), dim3(grid), dim3(BLOCK), 0, stream, a)
    if (fz && ad) {
        if (slot) TE_GL(MODE_SLOT, true, true);
        else TE_GL(MODE_CONTIG, true, true);
    } else if (fz) {
        if (slot) TE_GL(MODE_SLOT, true, false);
        else TE_GL(MODE_CONTIG, true, false);
    } else if (ad) {
        if (slot) TE_GL(MODE_SLOT, false, true);
        else TE_GL(MODE_CONTIG, false, true);
    } else {
        if (slot) TE_GL(MODE_SLOT, false, false);
        else TE_GL(MODE_CONTIG, false, false);
    }
#undef TE_GL
}

// --mtu-trunc placement (te_launch_t.static_mtu): the bytes each tile's records lose, as
// untrunc_packet cuts them (edit_packet.c:596-611): len > mtu + l2len -> caplen = len =
// l2len + mtu.  l2len is predicted from the frame's type field (14; 18 behind one
// 802.1Q / 802.1ad / QinQ tag).  The prediction only places the tiles: every tile checks
// its actual output total against it, and a mismatch (another L2 shape, an error, a
// record written unedited) sets *grow_bad and the host places the batch by scan instead.
// One wave per tile, its lanes over the tile's records (a thread walking a whole tile made
// ~100 dependent header loads per thread: 150 us for 4M IMIX records); each block takes 64
// tiles and leaves their block-local exclusive prefix in pre[] and their total in bsum[b].
__global__ void __launch_bounds__(256) te_mtu_tile_cut(const uint8_t *in, const te_tile_t *tiles,
                                                       const uint16_t *pkt_rel, uint32_t n, uint32_t mtu,
                                                       long long *pre, long long *bsum) {
    __shared__ long long c[64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t t0 = blockIdx.x * 64u;
    for (uint32_t j = w; j < 64u; j += 4u) {
        const uint32_t t = t0 + j;
        long long s = 0;
        if (t < n) {
            const te_tile_t tl = tiles[t];
            for (uint32_t k = lane; k < tl.npkt; k += 64u) {
                const uint8_t *r = in + tl.span_off + pkt_rel[tl.first_pkt + k];
                const uint32_t cap = ld32(r + 8), len = ld32(r + 12);
                uint32_t l2 = 14;
                if (cap >= 14) {
                    const uint32_t et = ((uint32_t)r[28] << 8) | r[29];
                    if (et == 0x8100u || et == 0x88a8u || et == 0x9100u) l2 = 18;
                }
                if (len > mtu + l2) s += (long long)cap - (long long)(l2 + mtu);
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) c[j] = s;
    }
    __syncthreads();
    if (w == 0) {
        const long long v = c[lane];
        long long x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long y = __shfl_up(x, o, 64);
            if ((int)lane >= o) x += y;
        }
        if (t0 + lane < n) pre[t0 + lane] = x - v;
        if (lane == 63) bsum[blockIdx.x] = x;
    }
}

// exclusive prefix of the block sums, in place (pre[n] = the total): one block walks them 4096
// at a time, four consecutive a thread (coalesced), a block scan of the threads' sums per step
__global__ void __launch_bounds__(1024) te_mtu_cut_scan(long long *pre, uint32_t n) {
    __shared__ long long wsum[16];
    __shared__ long long carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 4096u) {
        long long v[4], s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = base + 4u * tid + (uint32_t)k;
            v[k] = i < n ? pre[i] : 0ll;
            s += v[k];
        }
        long long x = s;  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long y = __shfl_up(x, o, 64);
            if ((int)lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        long long before = carry;
        for (uint32_t q = 0; q < w; ++q) before += wsum[q];
        before += x - s;  // this thread's exclusive prefix
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = base + 4u * tid + (uint32_t)k;
            if (i < n) pre[i] = before;
            before += v[k];
        }
        __syncthreads();
        if (tid == 1023) carry = before;  // (the last thread's running total is the step's end)
        __syncthreads();
    }
    if (tid == 0) pre[n] = carry;
}

// the block prefixes into the tiles' local prefixes; pre[n] = the batch total
__global__ void te_mtu_cut_add(long long *pre, const long long *bpre, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) pre[t] += bpre[t >> 6];
    else if (t == n) pre[n] = bpre[(n + 63u) >> 6];
}

// bsum: (n_tiles + 63) / 64 + 1 entries of scratch
extern "C" int te_mtu_cuts(const uint8_t *in, const te_tile_t *tiles, const uint16_t *pkt_rel, uint32_t n_tiles,
                           uint32_t mtu, long long *bsum, long long *pre, hipStream_t stream) {
    if (n_tiles == 0) return -1;
    const uint32_t nb = (n_tiles + 63u) / 64u;
    hipLaunchKernelGGL(te_mtu_tile_cut, dim3(nb), dim3(256), 0, stream, in, tiles, pkt_rel, n_tiles, mtu, pre, bsum);
    hipLaunchKernelGGL(te_mtu_cut_scan, dim3(1), dim3(1024), 0, stream, bsum, nb);
    hipLaunchKernelGGL(te_mtu_cut_add, dim3((n_tiles + 1u + 255u) / 256u), dim3(256), 0, stream, pre,
                       (const long long *)bsum, n_tiles);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ===========================================================================
// --fuzz-seed on the wave lane (te_launch_t.static_fz).  A record's RNG draw depends on how
// many records before it reach the fuzz step (te_fuzz_states), so the launch finds them
// first.  te_fuzz_reach reads each record's header and marks the records of the shape the
// wave lane edits -- Ethernet II with IPv4 IHL 5 or with IPv6 and TCP or UDP next, the
// network header captured: under the configs static_fz takes (no edit before the fuzz step
// but the en10mb decode and re-encode) such a record always reaches it (tcpedit.c:89-248:
// decode, encode, the IP header and L4 checks).  A tile holding any other record is listed,
// and the generic kernel's reach pass decides that tile.  For a marked record it also keeps
// what fuzzing() will look at (fuzzing.c:89-131) in one word, so the cut prediction reads no
// header again: caplen (bits 0-18), len < caplen (19), IPv6 (20), TCP (21), UDP (22), valid (31).
//
// Both kernels walk consecutive tiles a wave with every lane on a record (an IMIX tile of
// the lean budget holds ~14 records): the tiles' first records and span offsets go to LDS,
// and a lane finds its record's tile by a binary search there.  The reach kernel takes 16
// tiles a wave (a latency-bound gather: more waves in flight), the cut kernel 64 (its
// output is the per-64-tile layout te_mtu_cut_scan reads).
// ===========================================================================
constexpr uint32_t FZ_REACH_TILES = 16;
#ifndef FZ_REACH_U
#define FZ_REACH_U 4
#endif
constexpr uint32_t FZD_VALID = 1u << 31, FZD_LT = 1u << 19, FZD_V6 = 1u << 20, FZD_TCP = 1u << 21,
                   FZD_UDP = 1u << 22;

struct FzTiles {  // one wave's 64 tiles
    uint32_t fp[65];  // first record of each, and the end
    unsigned long long so[64];
};

// loads tiles [t0, t0 + G) into T (lane j: tile t0 + j); returns how many exist
template <uint32_t G = 64>
__device__ __forceinline__ uint32_t fz_load_tiles(const te_tile_t *tiles, uint32_t n, uint32_t t0, FzTiles &T,
                                                  uint32_t lane) {
    const uint32_t nt = n - t0 < G ? n - t0 : G;
    if (lane < nt) {
        const te_tile_t tl = tiles[t0 + lane];
        T.fp[lane] = tl.first_pkt;
        T.so[lane] = tl.span_off;
        if (lane == nt - 1) T.fp[nt] = tl.first_pkt + tl.npkt;
    }
    WK_LANES_SYNC();
    return nt;
}
// the tile (of the wave's nt) holding record r
__device__ __forceinline__ uint32_t fz_tile_of(const FzTiles &T, uint32_t nt, uint32_t r) {
    uint32_t lo = 0, hi = nt - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (T.fp[mid] <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void __launch_bounds__(256) te_fuzz_reach(const uint8_t *in, const te_tile_t *tiles, const uint16_t *pkt_rel,
                                                     uint32_t n, uint8_t *status, uint32_t *desc, uint32_t *list,
                                                     uint32_t *list_cnt, unsigned int *ticket) {
    __shared__ FzTiles TS[4];
    __shared__ uint32_t openb[4][2];
    if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t t0 = (blockIdx.x * 4u + w) * FZ_REACH_TILES;
    if (t0 >= n) return;  // (wave-uniform)
    FzTiles &T = TS[w];
    if (lane < 2) openb[w][lane] = 0;
    const uint32_t nt = fz_load_tiles<FZ_REACH_TILES>(tiles, n, t0, T, lane);
    const uint32_t r0 = T.fp[0], r1 = T.fp[nt];
    // FZ_REACH_U records a lane at once, each header read as three 16-byte loads from its
    // dword below caplen's field (the record offsets first, then every header load in flight
    // together: a record at a time waited out two dependent loads and 13 byte loads each)
    for (uint32_t rb = r0; rb < r1; rb += 64u * FZ_REACH_U) {
        uint32_t rr[FZ_REACH_U], rel[FZ_REACH_U];
#pragma unroll
        for (int k = 0; k < FZ_REACH_U; ++k) {
            rr[k] = umin32(rb + (uint32_t)lane + 64u * k, r1 - 1u);  // (past the end: the last record again)
            rel[k] = pkt_rel[rr[k]];
        }
        uint32_t q[FZ_REACH_U][12], sh[FZ_REACH_U], jt[FZ_REACH_U];
#pragma unroll
        for (int k = 0; k < FZ_REACH_U; ++k) {
            jt[k] = fz_tile_of(T, nt, rr[k]);
            const uint64_t a = T.so[jt[k]] + rel[k] + 8u;  // caplen's field
            sh[k] = (uint32_t)(a & 3u);
            const uint32_t *qa = (const uint32_t *)(in + (a & ~3ull));
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const uint4 v = *(const uint4 *)(qa + 4 * i);  // (the image has 64 bytes of slack past its end)
                q[k][4 * i] = v.x, q[k][4 * i + 1] = v.y, q[k][4 * i + 2] = v.z, q[k][4 * i + 3] = v.w;
            }
        }
#pragma unroll
        for (int k = 0; k < FZ_REACH_U; ++k) {
            const uint32_t r = rb + (uint32_t)lane + 64u * k;
            if (r >= r1) continue;
            // header bytes from caplen's field on: D[0] caplen, D[1] len, D[5] packet bytes 12..15,
            // D[7] packet bytes 20..23
            const uint32_t s8 = sh[k];
            const uint32_t cap = __builtin_amdgcn_alignbyte(q[k][1], q[k][0], s8);
            const uint32_t len = __builtin_amdgcn_alignbyte(q[k][2], q[k][1], s8);
            const uint32_t d5 = __builtin_amdgcn_alignbyte(q[k][6], q[k][5], s8);
            const uint32_t d7 = __builtin_amdgcn_alignbyte(q[k][8], q[k][7], s8);
            const uint32_t et = cap >= 14 ? ((d5 & 0xffu) << 8) | ((d5 >> 8) & 0xffu) : 0u;
            const uint32_t d14 = (d5 >> 16) & 0xffu, d20 = d7 & 0xffu, d23 = d7 >> 24;
            const bool v4 = et == 0x0800u && cap >= 34 && d14 == 0x45u;
            const bool v6 = et == 0x86DDu && cap >= 54 && (d20 == 6u || d20 == 17u);
            if (v4 || v6) {
                const uint32_t pr = v6 ? d20 : d23;
                status[r] = 1;
                desc[r] = FZD_VALID | cap | (len < cap ? FZD_LT : 0u) | (v6 ? FZD_V6 : 0u) | (pr == 6u ? FZD_TCP : 0u) |
                          (pr == 17u ? FZD_UDP : 0u);
            } else {
                desc[r] = 0u;
                atomicOr(&openb[w][jt[k] >> 5], 1u << (jt[k] & 31u));
            }
        }
    }
    WK_LANES_SYNC();
    if (lane < nt && ((openb[w][lane >> 5] >> (lane & 31u)) & 1u)) list[atomicAdd(list_cnt, 1u)] = t0 + lane;
}

// the bytes each tile's records lose to fuzzing() (DROP: the whole record; REDUCE: its tail),
// from the reach flags, the RNG states and te_fuzz_reach's words (the records of a listed tile
// read their headers), laid out as te_mtu_tile_cut's: per 64 tiles a local exclusive prefix in
// pre[] and the total in bsum[].  With no edit before the fuzz step but the en10mb decode and
// re-encode, fuzzing() sees the input bytes, so this is its choice (every tile checks its
// output total against it).
__global__ void __launch_bounds__(256) te_fuzz_tile_cut(const uint8_t *in, const te_tile_t *tiles,
                                                        const uint16_t *pkt_rel, uint32_t n, const uint8_t *status,
                                                        const uint32_t *states, const uint32_t *desc,
                                                        const te_dev_cfg_t *cfg, long long *pre, long long *bsum) {
    __shared__ FzTiles TS[4];
    __shared__ uint32_t cut[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * 4u + w, t0 = g * 64u;
    if (t0 >= n) return;  // (wave-uniform)
    FzTiles &T = TS[w];
    cut[w][lane] = 0;
    const uint32_t nt = fz_load_tiles(tiles, n, t0, T, lane);
    const uint32_t factor = cfg->fuzz_factor;
    const uint32_t r0 = T.fp[0], r1 = T.fp[nt];
    // FZ_REACH_U records a lane at once, their flag, state and word loaded together (a record
    // at a time waited for the flag, then for the state)
    for (uint32_t rb = r0; rb < r1; rb += 64u * FZ_REACH_U) {
    uint32_t fl_[FZ_REACH_U], st_[FZ_REACH_U], dw_[FZ_REACH_U];
#pragma unroll
    for (int k = 0; k < FZ_REACH_U; ++k) {
        const uint32_t rk = umin32(rb + (uint32_t)lane + 64u * k, r1 - 1u);
        fl_[k] = status[rk];
        st_[k] = states[rk];
        dw_[k] = desc[rk];
    }
#pragma unroll
    for (int k = 0; k < FZ_REACH_U; ++k) {
        const uint32_t r = rb + (uint32_t)lane + 64u * k;
        if (r >= r1 || !(fl_[k] & 1u)) continue;
        uint32_t st = st_[k];
        const uint32_t rnd = tcpr_random_dev(st);
        if (rnd % factor) continue;
        const uint32_t dw = dw_[k];
        FzPlan f;
        uint32_t cap;
        if (dw & FZD_VALID) {
            cap = dw & 0x7ffffu;
            const int l3 = (dw & FZD_V6) ? 54 : 34, adj = (dw & FZD_TCP) ? 20 : (dw & FZD_UDP) ? 8 : 0;
            f = fuzz_plan_l4(rnd, l3 + adj, l3 - adj, cap, (dw & FZD_LT) ? 0u : cap);
        } else {
            const uint32_t j = fz_tile_of(T, nt, r);
            const uint8_t *rec = in + T.so[j] + pkt_rel[r];
            cap = ld32(rec + 8);
            f = fuzz_plan(rec + 16, cap, ld32(rec + 12), cap, *cfg, rnd);
        }
        if (f.cut) atomicAdd(&cut[w][fz_tile_of(T, nt, r)], f.nl ? cap - f.nl : 16u + cap);
    }
    }
    WK_LANES_SYNC();
    const long long v = lane < nt ? (long long)cut[w][lane] : 0ll;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(x, o, 64);
        if ((int)lane >= o) x += y;
    }
    if (lane < nt) pre[t0 + lane] = x - v;
    if (lane == 63) bsum[g] = x;
}

// static_fz's prelude: the reach (header kernel + the generic reach pass over the tiles it
// listed), the RNG states, the placement prediction (tcut)
static int fuzz_wave_prelude(const te_launch_t *L, const LaunchArgs &a, hipStream_t stream) {
    if (!L->fuzz_states || !L->fuzz_blk || !L->fuzz_words || !L->fz_list || !L->tcut || !L->tcut_raw ||
        L->n_pkts == 0 || L->n_tiles == 0)
        return -1;
    uint32_t *cnt = L->fz_list + L->n_tiles, *desc = cnt + 1;
    const uint32_t ng = (L->n_tiles + 63u) / 64u;  // groups of 64 tiles, a wave each
    const uint32_t nr = (L->n_tiles + FZ_REACH_TILES - 1) / FZ_REACH_TILES;  // the reach kernel's groups
    if (hipMemsetAsync(cnt, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    hipLaunchKernelGGL(te_fuzz_reach, dim3((nr + 3u) / 4u), dim3(256), 0, stream, L->in, L->tiles, L->pkt_rel,
                       L->n_tiles, L->status, desc, L->fz_list, cnt, L->ticket);
    LaunchArgs pa = a;
    pa.tile_list = L->fz_list;
    pa.list_cnt = cnt;
    pa.counters_next = nullptr;
    pa.fuzz_mode = TE_FUZZ_PROBE;
    launch_generic(true, false, false, resident_blocks(0), stream, pa);
    const uint32_t nblk = (L->n_pkts + FZ_PER_BLOCK - 1) / FZ_PER_BLOCK;
    hipLaunchKernelGGL(te_fuzz_count, dim3(nblk), dim3(FZ_BLOCK), 0, stream, (const uint8_t *)L->status, L->n_pkts,
                       L->fuzz_blk);
    hipLaunchKernelGGL(te_fuzz_scan, dim3(1), dim3(1024), 0, stream, L->fuzz_blk, nblk, L->fuzz_words, 1);
    hipLaunchKernelGGL(te_fuzz_states, dim3(nblk), dim3(FZ_BLOCK), 0, stream, (const uint8_t *)L->status, L->n_pkts,
                       (const uint32_t *)L->fuzz_blk, (const uint32_t *)L->fuzz_words, L->fuzz_states);
    long long *pre = (long long *)L->tcut, *bsum = (long long *)L->tcut_raw;
    hipLaunchKernelGGL(te_fuzz_tile_cut, dim3((ng + 3u) / 4u), dim3(256), 0, stream, L->in, L->tiles, L->pkt_rel,
                       L->n_tiles, (const uint8_t *)L->status, (const uint32_t *)L->fuzz_states,
                       (const uint32_t *)desc, L->cfg, pre, bsum);
    hipLaunchKernelGGL(te_mtu_cut_scan, dim3(1), dim3(1024), 0, stream, bsum, ng);
    hipLaunchKernelGGL(te_mtu_cut_add, dim3((L->n_tiles + 1u + 255u) / 256u), dim3(256), 0, stream, pre,
                       (const long long *)bsum, L->n_tiles);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int te_launch_edit(te_launch_t *L, hipStream_t stream) {
    LaunchArgs a;
    fill_args(a, L);
    hipError_t e;
    const bool fast = L->fast &&
                      ((L->static_off && !L->slot_layout) || L->static_grow || L->static_shrink || L->static_mtu ||
                       L->static_fz) &&
                      L->n_tiles > 0;
    if (L->win) {  // window mode: the wave lane finds its records; then the chain check
        if (!L->cfg_host || L->in_swapped || L->in_nsec || L->dirbits || L->nwin == 0) return -1;
        FastArgs f;
        memset(&f, 0, sizeof f);
        f.cfg = L->cfg;
        f.portlut = L->portlut;
        f.in = L->in;
        f.out = L->out;
        f.status = L->status;
        f.list_cnt_next = L->list_cnt + 1;
        f.counters_next = (unsigned long long *)L->counters_next;
        f.ws_zero = (unsigned long long *)L->ws_zero;
        f.out_base = L->out_base;
        f.rec0 = L->rec0;
        f.fixed_dir = L->fixed_dir;
        f.v6_ok = (uint32_t)L->fast_v6;
        f.stream = (uint32_t)L->stream;
        f.slots = (unsigned long long *)L->slots;
        const te_dev_cfg_t *ch = L->cfg_host;
        f.seed_sw = __builtin_bswap32(ch->seed);
        f.seed_on = ch->seed != 0;
        f.skip_bcast = ch->skip_broadcast != 0;
        f.win_len = L->win_len;
        f.win_entry = L->win_entry;
        f.win_entry_ptr = L->win_entry_ptr;
        f.win_entry_sub = L->win_entry_sub;
        f.win_base = L->win_base;
        f.win_limit = L->win_limit;
        f.nwin = L->nwin;
        f.w_entry = L->w_entry;
        f.w_exit = L->w_exit;
        f.w_flags = L->w_flags;
        f.win_bad = L->win_bad;
        f.win_tot = (unsigned long long *)L->win_tot;
        const uint32_t want = fast_feat(ch);
        int wk = -1;
        for (int k = 0; k < (int)(sizeof(win_inst) / sizeof(win_inst[0])) && wk < 0; ++k)
            if ((want & ~win_inst[k].feat) == 0 && ((want ^ win_inst[k].feat) & TE_FF_INCR) == 0) wk = k;
        if (wk < 0) return -1;
        if (!win_inst[wk].grid) {
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, win_inst[wk].fn, WKB, 0) != hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            win_inst[wk].grid = cu_count() * per_cu;
        }
        int grid = win_inst[wk].grid;
        const uint32_t need = (L->nwin + WK_NW - 1) / WK_NW;
        if ((uint32_t)grid > need) grid = (int)need;
        {  // TCPEDIT_HIP_WIN_BALANCE=1: equal rounds of windows, as the wave lane's tiles
            static int wb = -1;
            if (wb < 0) wb = getenv("TCPEDIT_HIP_WIN_BALANCE") ? atoi(getenv("TCPEDIT_HIP_WIN_BALANCE")) != 0 : 0;
            if (wb && grid > 0) {
                const uint32_t wv = (uint32_t)grid * WK_NW, rounds = (L->nwin + wv - 1) / wv;
                const uint32_t bal = ((L->nwin + rounds - 1) / rounds + WK_NW - 1) / WK_NW;
                if (bal >= 1 && bal < (uint32_t)grid) grid = (int)bal;
            }
        }
        if (grid < 1 || ((L->out_base - L->rec0) & 15)) return -1;
        // (the verdict words: zeroed by the window kernel itself, which never writes them)
        if (L->ev_k0 && hipEventRecord((hipEvent_t)L->ev_k0, stream) != hipSuccess) return -1;
        {
            void *args[] = {&f};
            if (hipLaunchKernel(win_inst[wk].fn, dim3(grid), dim3(WKB), args, 0, stream) != hipSuccess) return -1;
        }
        WinTail wt;
        wt.acc = (unsigned long long *)L->win_acc;
        wt.slots = (const unsigned long long *)L->slots;
        wt.nslots = (uint32_t)grid;
        wt.ncheck = (L->nwin + 255) / 256;
        wt.prev_out = L->win_prev_out && L->win_entry_ptr ? L->win_prev_out : nullptr;
        wt.out = L->out;
        wt.head_max = L->win_head_max;
        wt.org = L->win_org ? L->win_org : 24;
        const uint32_t nx = (wt.acc ? 1u : 0u) + (wt.prev_out ? WIN_HEAD_BLOCKS : 0u);
        hipLaunchKernelGGL(te_win_check, dim3(wt.ncheck + nx), dim3(256), 0, stream, f,
                           (unsigned long long *)L->win_tot, wt);
        if (L->ev_k1 && hipEventRecord((hipEvent_t)L->ev_k1, stream) != hipSuccess) return -1;
        L->out_fgrid = grid;
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (fast && !L->generic_only) {
        if (L->static_fz && fuzz_wave_prelude(L, a, stream) != 0) return -1;
        // the fast kernel zeroes the generic kernel's words itself: no memset launch
        FastArgs f;
        f.cfg = L->cfg;
        f.portlut = L->portlut;
        f.dirbits = L->dirbits;
        f.dirbits_len = L->dirbits_len;
        f.pkt_base = L->pkt_base;
        f.in = L->in;
        f.tiles = L->tiles;
        f.pkt_rel = L->pkt_rel;
        f.out = L->out;
        f.status = L->status;
        f.tile_list = L->tile_list;
        f.list_cnt = L->list_cnt + (L->parity & 1);
        f.list_cnt_next = L->list_cnt + ((L->parity & 1) ^ 1);
        f.counters = (unsigned long long *)L->counters;
        f.ws_zero = (unsigned long long *)L->ws_zero;
        f.out_base = L->out_base;
        f.rec0 = L->rec0;
        f.n_tiles = L->n_tiles;
        f.fixed_dir = L->fixed_dir;
        f.in_swapped = L->in_swapped;
        f.in_nsec = L->in_nsec;
        f.v6_ok = (uint32_t)L->fast_v6;
        f.stream = (uint32_t)L->stream;
        f.slots = (unsigned long long *)L->slots;
        f.counters_next = (unsigned long long *)L->counters_next;
        const te_dev_cfg_t *ch = L->cfg_host;
        if (!ch) return -1;
        f.seed_sw = __builtin_bswap32(ch->seed);
        f.seed_on = ch->seed != 0;
        f.skip_bcast = ch->skip_broadcast != 0;
        const bool grow = L->static_grow != 0;
        if (grow) {  // the pushed {TPID, TCI} of an untagged frame, as dlt_en10mb_encode builds it
            uint16_t tci = __builtin_bswap16((uint16_t)(ch->vlan_tag & 0x0fffu));
            if (ch->vlan_pri < 255) tci = (uint16_t)(tci + __builtin_bswap16((uint16_t)(ch->vlan_pri << 13)));
            if (ch->vlan_cfi < 255) tci = (uint16_t)(tci + __builtin_bswap16((uint16_t)(ch->vlan_cfi << 12)));
            f.vlan_tag_word = (uint32_t)__builtin_bswap16((uint16_t)ch->vlan_proto) | ((uint32_t)tci << 16);
        } else {
            f.vlan_tag_word = 0;
        }
        f.mtu = L->static_mtu ? L->mtu : 0u;
        f.tcut = (const long long *)L->tcut;
        f.grow_bad = L->grow_bad;
        f.fz_state = L->static_fz ? L->fuzz_states : nullptr;
        f.fz_factor = ch->fuzz_factor ? ch->fuzz_factor : 1u;
        if ((L->static_mtu || L->static_fz) && (!L->tcut || L->fast_kind != TE_FAST_WAVE)) return -1;
        const void *wfn = nullptr;
        const int wk = wave_pick(fast_feat(ch) | (L->wk_small ? TE_FF_SMALL : 0u), grow ? SZ_GROW
                                                : L->static_mtu ? SZ_MTU
                                                : L->static_fz  ? SZ_FUZZ
                                                                : L->static_shrink);
        if (wk < 0) return -1;
        wfn = wave_inst[wk].fn;
        const bool wave = L->fast_kind == TE_FAST_WAVE;
        int fgrid = wave ? wave_inst_grid(wk) : te_fast_grid();
        if (fgrid < 1) return -1;
        const uint32_t need = wave ? (L->n_tiles + WK_NW - 1) / WK_NW : L->n_tiles;
        if ((uint32_t)fgrid > need) fgrid = (int)need;
        if (wave && wave_balance()) {
            const uint32_t wv = (uint32_t)fgrid * WK_NW, rounds = (L->n_tiles + wv - 1) / wv;
            const uint32_t bal = ((L->n_tiles + rounds - 1) / rounds + WK_NW - 1) / WK_NW;
            if (bal >= 1 && bal < (uint32_t)fgrid) fgrid = (int)bal;
        }
        if (wave) {  // (diagnostics: TCPEDIT_HIP_WAVE_GRID_SUB=k launches k blocks fewer)
            static int sub = -1, rot = -1;
            if (sub < 0) sub = getenv("TCPEDIT_HIP_WAVE_GRID_SUB") ? atoi(getenv("TCPEDIT_HIP_WAVE_GRID_SUB")) : 0;
            if (sub > 0 && sub < fgrid) fgrid -= sub;
            // a grid that is a multiple of the 8 XCDs deals each XCD the same tile stripes every
            // round: C5 at 1,024 blocks 0.630, at 1,023 0.645-0.667 (A/B); one block fewer there
            // (C3, C4, hdr, vdel: no change either way; TCPEDIT_HIP_WAVE_ROTATE=0 keeps it)
            if (rot < 0) rot = getenv("TCPEDIT_HIP_WAVE_ROTATE") ? atoi(getenv("TCPEDIT_HIP_WAVE_ROTATE")) != 0 : 1;
            if (rot && fgrid > 8 && fgrid % 8 == 0) {  // (only where the rounds stay as many)
                const uint32_t w1 = (uint32_t)fgrid * WK_NW, w2 = w1 - WK_NW;
                if ((L->n_tiles + w1 - 1) / w1 == (L->n_tiles + w2 - 1) / w2) fgrid -= 1;
            }
        }
        if (wave && (!L->slots || ((L->out_base - L->rec0) & 15)))
            return -1;  // the wave lane stores whole 16-byte chunks at input offsets + a multiple of 16
        if (L->ev_k0 && hipEventRecord((hipEvent_t)L->ev_k0, stream) != hipSuccess) return -1;
        if (wave)
        {
            void *args[] = {&f};
            if (hipLaunchKernel(wfn, dim3(fgrid), dim3(WKB), args, 0, stream) != hipSuccess) return -1;
        }
        else
            hipLaunchKernelGGL(te_fast_tiles, dim3(fgrid), dim3(FKB), 0, stream, f);
        if (L->ev_k1 && hipEventRecord((hipEvent_t)L->ev_k1, stream) != hipSuccess) return -1;
        if (hipGetLastError() != hipSuccess) return -1;
        L->out_fgrid = fgrid;
        // after the wave lane the host leaves the generic pass out when this batch's
        // previous run listed no tile (and runs it, generic_only, if a run ever does)
        if (L->skip_generic) return 0;
    }
    if (fast) {  // the generic kernel redoes only the tiles the fast lane listed
        a.tile_list = L->tile_list;
        a.list_cnt = L->list_cnt + (L->parity & 1);
        a.counters_next = (unsigned long long *)L->counters_next;
        if (L->static_fz) {  // ... fuzzing them with the states the prelude drew
            a.fuzz_mode = TE_FUZZ_APPLY;
            a.fuzz_state = L->fuzz_states;
        }
    } else {
        // one memset per launch: error words, ticket, counters, look-back granules
        e = hipMemsetAsync(L->zero_region, 0, L->zero_bytes, stream);
        if (e != hipSuccess) return -1;
        if (L->n_tiles == 0) return 0;
    }
    // after the fast lane the host may pass a smaller grid (the tiles the previous run of
    // this batch listed): the loop below takes tickets, so any grid >= 1 edits every tile
    const int res = resident_blocks(L->slot_layout);
    int grid = L->grid > 0 && L->grid < res ? L->grid : res;
    if ((uint32_t)grid > L->n_tiles) grid = (int)L->n_tiles;
    if (!fast && jnpr_prepare(L, a, stream) != 0) return -1;
    if (L->fuzz_states && !fast) {
        // --fuzz-seed: reach pass, per-record RNG states, then the edit pass below
        if (!L->fuzz_blk || !L->fuzz_words || L->n_pkts == 0) return -1;
        a.fuzz_mode = TE_FUZZ_PROBE;
        launch_generic(true, L->any_dec != 0, L->slot_layout != 0, grid, stream, a);
        const uint32_t nblk = (L->n_pkts + FZ_PER_BLOCK - 1) / FZ_PER_BLOCK;
        hipLaunchKernelGGL(te_fuzz_count, dim3(nblk), dim3(FZ_BLOCK), 0, stream, (const uint8_t *)L->status,
                           L->n_pkts, L->fuzz_blk);
        hipLaunchKernelGGL(te_fuzz_scan, dim3(1), dim3(1024), 0, stream, L->fuzz_blk, nblk, L->fuzz_words,
                           L->fuzz_probe_only ? 0 : L->q18_only ? 2 : 1);
        if (L->fuzz_probe_only) return hipGetLastError() == hipSuccess ? 0 : -1;
        hipLaunchKernelGGL(te_fuzz_states, dim3(nblk), dim3(FZ_BLOCK), 0, stream, (const uint8_t *)L->status,
                           L->n_pkts, (const uint32_t *)L->fuzz_blk, (const uint32_t *)L->fuzz_words,
                           L->fuzz_states);
        if (hipGetLastError() != hipSuccess) return -1;
        e = hipMemsetAsync(L->zero_region, 0, L->zero_bytes, stream);  // the reach pass took tickets
        if (e != hipSuccess) return -1;
        a.fuzz_mode = TE_FUZZ_APPLY;
        a.fuzz_state = L->fuzz_states;
    }
    if (!fast && l2carry_prepare(L, a, stream, grid) != 0) return -1;
    if (L->q18_only) return L->fuzz_states && L->l2carry && hipGetLastError() == hipSuccess ? 0 : -1;
    const bool ev = !fast && L->ev_k0;  // without the fast lane this kernel is the edit kernel
    if (ev && hipEventRecord((hipEvent_t)L->ev_k0, stream) != hipSuccess) return -1;
    launch_generic(a.fuzz_mode != TE_FUZZ_OFF, L->any_dec != 0, L->slot_layout != 0, grid, stream, a);
    if (ev && hipEventRecord((hipEvent_t)L->ev_k1, stream) != hipSuccess) return -1;
    if (!fast && L->l2carry)  // the last record's value, for the next launch (the Q8 replay reads the array)
        hipLaunchKernelGGL(te_l2carry_save, dim3(1), dim3(64), 0, stream, (const unsigned long long *)L->l2carry,
                           L->n_pkts, L->l2carry_word);
    if (!fast && L->jscan)  // the launch's last whole Juniper decode, for the next launch
        hipLaunchKernelGGL(te_jnpr_save, dim3(1), dim3(64), 0, stream, (const unsigned long long *)L->jscan,
                           L->jstates, L->n_pkts, L->jctx, (te_jctx_t *)nullptr);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : -1;
}

extern "C" uint32_t te_win_bytes(void) { return (uint32_t)WIN_WN; }


extern "C" int te_launch_packet_server(const te_srv_launch_t *S, hipStream_t stream) {
    hipLaunchKernelGGL(te_packet_server, dim3(1), dim3(BLOCK), 0, stream, *S);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
