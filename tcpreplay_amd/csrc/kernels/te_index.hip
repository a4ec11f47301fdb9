// te_index.hip -- the record index on the device (index -> edit -> scan
// -> compaction; 7 hard part 5: chunked speculation).
//
// libpcap reads a capture as a chain of records, each header saying where the next one
// starts (tcprewrite.c:289 pcap_next).  The host walks that chain (te_api.c walk_range);
// here it is found in parallel, speculatively, and checked exactly, in four launches with
// no window ever waiting on another:
//   * te_index_count, a wave per window: the capture is cut into windows of W = 64 S bytes
//     (each owning W - OL S bytes, the first OL sub-windows being the previous window's),
//     every window into 64 sub-windows of S bytes, one lane each.  The record discovery is
//     te_window.hpp find_window (shared with the edit's window mode): the wave stages its
//     window into LDS with coalesced 16-byte loads; a lane guesses the first record start
//     in its sub-window from the zero-byte mask of its dwords (a header has zero bytes at
//     +11 and +15 -- caplen, len <= 262144 -- and at +7 for a microsecond capture) and the
//     header behind the guess, walks its records, and the guesses are reconciled exactly (a
//     lane's guess must be where the nearest earlier guessing lane's walk ended: ballots and
//     bit searches, Jacobi rounds, a serial lane loop as the last resort).  The wave cuts
//     its records into wave-lane tiles as walk_range cuts them (byte budget, 64 records,
//     solo and huge records; a tile never spans two windows) and writes its facts (entry,
//     exit, chain flags, records | tiles, huge-record scratch bytes) and its cut to a
//     per-window scratch area;
//   * te_index_part (a block of 1,024 windows) and te_index_scan (one block): exclusive
//     scans of (records | tiles), scratch bytes and the last window with a record, libpcap's
//     first stop, the totals;
//   * te_index_write, a wave per window: the window's tiles and record offsets at its global
//     bases, and the chain check -- a window's first record must be where the chain left the
//     nearest earlier window a record starts in (window kE starts at the known first record),
//     and a window without one must be passed over whole.  A miss sets IDX_T_BAD and the
//     caller keeps the host walk's index, which is exact.
//   (A single-pass version with a decoupled look-back over windows and a serial finishing
//   check cost ~50 ns a window: 0.84 ms on C2.)
// libpcap's ends are kept: an oversize record (caplen > 262144) or a truncated one ends
// the chain; a record with len > 262144, len 0 or caplen 0 ends it with safe_pcap_next's
// exit (src/common/utils.c:136-156).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "te_index.h"
#include "te_window.hpp"

namespace {
using namespace tew;

constexpr int IB = 256;                      // threads per block: 4 windows in flight
constexpr int IWAVES = IB / IW;
constexpr int REC_BITS = 36;                 // a window's (records | tiles << 36)
constexpr u64 REC_MASK = (1ull << REC_BITS) - 1;

// one wave's LDS: the staged window, its record offsets, per-record tile starts, tile starts
template <int S>
struct alignas(16) WinLds {
    static constexpr int W = IW * S;
    static constexpr int MAXR = W / 16;      // records starting in a window, at most
    u32 img[(W + 48) / 4];                   // bytes [A0, A0 + W + 48): A0 = window start & ~15
    u32 rel[MAXR + 1];                       // record offset from the window start (+ end of the last)
    u16 tsi[MAXR];                           // the record's tile's first record
    u16 tst[MAXR + 1];                       // tile start records (+ nrec)
    u64 pfx;                                 // the window's exclusive (records | tiles) prefix
};

// Window geometry: window k owns the record starts in [ws, we), ws = base + k WN.  Its wave
// stages [ws - O, we + 16): the O = OL S bytes before the window are the first OL lanes'
// sub-windows, whose only job is to establish the chain entering ws (a guess there that is
// not a record start is corrected as the chain runs on, or leaves the window before ws).
// what the scan needs of a window
struct Facts {
    u64 went, wexit;  // where the chain enters and leaves it (IDX_NONE: no record starts here)
    u64 scr;          // scratch bytes of its huge records
    u32 nrec, ntile, flags;
};
template <int S, int OL>
__device__ __forceinline__ Facts count_window(const IdxArgs &a, WinLds<S> &M, u32 k) {
    const int lane = threadIdx.x & 63;
    const tew::Found fw = tew::find_window<S, OL>(a, M.img, M.rel, k);
    const u64 ws = fw.ws, went = fw.went, wexit = fw.wexit;
    const u32 wstop = fw.wstop, nrec = fw.nrec;
    const bool anytrim = fw.anytrim;

    // ---- the tile cut: one ballot per tile ----
    u32 ntile = 0;
    for (u32 s = 0; s < nrec;) {
        const u32 i = s + lane;
        const bool v = i < nrec && lane < (int)a.max_pkts;
        const u32 r = v ? M.rel[i] : 0, r1 = v ? M.rel[i + 1] : 0;
        const u32 cl = r1 - r - 16;
        const u32 g = (u32)((ws + r) & 15);
        bool huge = v && !TE_CONTIG_FITS_IN(g, 16 + cl, a.budget);
        const bool solo = huge && TE_CONTIG_FITS(g, 16 + cl);
        huge = huge && !solo;
        const u32 rs = __shfl(r, 0);
        const u64 t0 = ws + rs;
        const bool fits = v && TE_CONTIG_FITS_IN((u32)(t0 & 15), r1 - rs, a.budget);
        const bool lone0 = __shfl((int)(huge || solo), 0) != 0;
        const u64 brk = __ballot(lane > 0 && (!v || huge || solo || !fits));
        const u32 len = lone0 ? 1u : (brk ? (u32)__builtin_ctzll(brk) : 64u);
        if (lane == 0) M.tst[ntile] = (u16)s;
        if (lane < (int)len) M.tsi[i] = (u16)s;
        ++ntile;
        s += len;
    }
    if (lane == 0) M.tst[ntile] = (u16)nrec;
    asm volatile("" ::: "memory");

    // ---- the window's facts for the scan, and its cut for the write pass ----
    // (huge records -- larger than a tile -- get an HBM scratch slot: its bytes here, the
    // slot's offset from the scan of every window's bytes)
    u64 scr = 0;
    for (u32 t = lane; t < ntile; t += IW) {
        const u32 s0 = M.tst[t], s1 = M.tst[t + 1];
        const u32 span = M.rel[s1] - M.rel[s0];
        const u32 g = (u32)((ws + M.rel[s0]) & 15);
        if (s1 - s0 == 1 && !TE_CONTIG_FITS_IN(g, span, a.budget) && !TE_CONTIG_FITS(g, span))
            scr += ((u64)TE_SLOT_BYTES_OF(g, span - 16) + TE_LDS_FRONT + 64 + 255) & ~255ull;
        if (t < (u32)IDX_MAXR) ((uint2 *)a.t_tile)[(u64)k * IDX_MAXR + t] = make_uint2(M.rel[s0], s0 | (s1 - s0) << 16);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) scr += __shfl_xor(scr, o, 64);
    for (u32 i = lane; i < nrec; i += IW)
        if (i < (u32)IDX_MAXR) a.t_prel[(u64)k * IDX_MAXR + i] = (u16)(M.rel[i] - M.rel[M.tsi[i]]);
    return Facts{went, wexit, scr, nrec, ntile, wstop | (anytrim ? IDX_TRIM : 0u)};
}

// ---- the scan, in two levels: te_index_part (a block of SB windows, one a thread) leaves
// each window's in-block exclusive prefixes of (records | tiles) and scratch bytes and the
// nearest earlier window with a record in the block, and the block's totals (a Part);
// te_index_scan (one block) scans the Parts, finds libpcap's first stop and writes the
// totals.  The write pass checks the chain window by window.
constexpr int SB = IDX_SB;
constexpr long long NO_STOP = 0x7fffffffffffffffll;
struct Part {           // a block's totals, then (te_index_scan) their exclusive prefixes
    u64 agg, scr;
    long long lastrec;  // the last window at or after kE with a record (-1: none)
    long long stop;     // the first window where the chain stops (NO_STOP: none)
};
static_assert(sizeof(Part) == IDX_PART_BYTES, "te_index.h sizes the scan blocks' records");
constexpr u32 STOPS = IDX_STOP | IDX_ERROR | IDX_END;
constexpr u64 WNB = (u64)IW * TE_IDX_S - (u64)TE_IDX_OL * TE_IDX_S;  // bytes a window owns
__device__ __forceinline__ u32 idx_kE(const IdxArgs &a, u64 &entry) {
    entry = a.entry_ptr ? *(const volatile u64 *)a.entry_ptr - a.entry_sub : a.entry;
    return (u32)((entry - a.base) / WNB);
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl(T x, Op op) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= o) x = op(x, y);
    }
    return x;
}
// exclusive block scan (SB threads, thread order); `total` = the whole block's
template <typename T, typename Op>
__device__ __forceinline__ T block_ex(T v, T ident, Op op, T *wsum, T &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const T inc = wave_incl(v, op);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    T base = ident, tot = ident;
#pragma unroll
    for (int w = 0; w < SB / 64; ++w) {
        const T x = wsum[w];
        if (w < wid) base = op(base, x);
        tot = op(tot, x);
    }
    __syncthreads();
    total = tot;
    T ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = ident;
    return op(base, ex);
}
struct SumOp { __device__ u64 operator()(u64 x, u64 y) const { return x + y; } };
struct MaxOp { __device__ long long operator()(long long x, long long y) const { return x > y ? x : y; } };
struct MinOp { __device__ long long operator()(long long x, long long y) const { return x < y ? x : y; } };

template <int S, int OL>
__global__ __launch_bounds__(IB) void te_index_count(IdxArgs a) {
    __shared__ WinLds<S> L[IWAVES];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u32 k = blockIdx.x * IWAVES + (u32)wv;  // windows are independent here: no order
    if (k >= a.nwin) return;
    const Facts f = count_window<S, OL>(a, L[wv], k);
    if (lane == 0) {
        a.w_entry[k] = f.went;
        a.w_exit[k] = f.wexit;
        a.w_flags[k] = f.flags;
        a.w_agg[k] = (u64)f.nrec | ((u64)f.ntile << REC_BITS);
        a.w_scr[k] = f.scr;
    }
}

__global__ __launch_bounds__(SB) void te_index_part(IdxArgs a) {
    __shared__ u64 ws64[SB / 64];
    __shared__ long long wsll[SB / 64];
    u64 entry;
    const u32 kE = idx_kE(a, entry);
    const u32 q = blockIdx.x * SB + threadIdx.x;
    const bool in = q < a.nwin;
    const u64 eq = in ? a.w_entry[q] : IDX_NONE;
    const u32 fl = in ? a.w_flags[q] : 0u;
    const u64 agg = in ? a.w_agg[q] : 0ull, scr = in ? a.w_scr[q] : 0ull;
    const long long rec = in && q >= kE && eq != IDX_NONE ? (long long)q : -1ll;
    const long long stp = eq != IDX_NONE && (fl & STOPS) ? (long long)q : NO_STOP;
    Part P;
    const u64 xa = block_ex(agg, (u64)0, SumOp(), ws64, P.agg);
    const u64 xs = block_ex(scr, (u64)0, SumOp(), ws64, P.scr);
    const long long xr = block_ex(rec, -1ll, MaxOp(), wsll, P.lastrec);
    (void)block_ex(stp, NO_STOP, MinOp(), wsll, P.stop);
    if (in) {
        a.w_pfx[q] = xa;
        a.w_sbase[q] = xs;
        a.w_prev[q] = xr;
    }
    if (threadIdx.x == 0) ((Part *)a.parts)[blockIdx.x] = P;
}

__global__ __launch_bounds__(SB) void te_index_scan(IdxArgs a) {
    __shared__ u64 ws64[SB / 64];
    __shared__ long long wsll[SB / 64];
    u64 entry;
    const u32 kE = idx_kE(a, entry);
    const u32 G = (a.nwin + SB - 1) / SB;
    Part *parts = (Part *)a.parts;
    u64 ca = 0, cs = 0;
    long long cr = -1, cstop = NO_STOP;
    for (u32 g0 = 0; g0 < G; g0 += SB) {  // (one round up to SB^2 windows)
        const u32 g = g0 + threadIdx.x;
        const bool in = g < G;
        const Part P = in ? parts[g] : Part{0, 0, -1, NO_STOP};
        u64 ta, ts;
        long long tr, tst;
        const u64 xa = block_ex(P.agg, (u64)0, SumOp(), ws64, ta);
        const u64 xs = block_ex(P.scr, (u64)0, SumOp(), ws64, ts);
        const long long xr = block_ex(P.lastrec, -1ll, MaxOp(), wsll, tr);
        (void)block_ex(P.stop, NO_STOP, MinOp(), wsll, tst);
        if (in) parts[g] = Part{ca + xa, cs + xs, xr > cr ? xr : cr, NO_STOP};
        ca += ta;
        cs += ts;
        cr = tr > cr ? tr : cr;
        cstop = tst < cstop ? tst : cstop;
    }
    if (threadIdx.x) return;
    const bool stopped = cstop != NO_STOP;
    const u32 last = stopped ? (u32)cstop : a.nwin - 1;  // windows past the chain's end do not count
    u64 tot, scr, end;
    u32 fl_last = 0;
    if (!stopped) {  // the whole capture's totals; the chain ends in the last window with a record
        tot = ca;
        scr = cs;
        end = cr >= (long long)kE ? a.w_exit[cr] : IDX_NONE;
    } else {
        const Part &L = parts[last / SB];
        tot = L.agg + a.w_pfx[last] + a.w_agg[last];  // inclusive (records | tiles) through `last`
        scr = L.scr + a.w_sbase[last] + a.w_scr[last];
        end = a.w_exit[last];  // (a window that stops the chain has a record)
        fl_last = a.w_flags[last];
    }
    a.totals[IDX_T_RECS] = tot & REC_MASK;
    a.totals[IDX_T_TILES] = tot >> REC_BITS;
    a.totals[IDX_T_SCRATCH] = scr;
    a.totals[IDX_T_WINDOWS] = last + 1;
    a.totals[IDX_T_STOP] = stopped ? (fl_last & STOPS) : 0;
    a.totals[IDX_T_END] = end == IDX_NONE ? entry : end;
    a.totals[IDX_T_BYTES] = (a.totals[IDX_T_END] - entry) + (u64)a.growth * (tot & REC_MASK);
    // the record the chain stopped at: the one after the stopping window's last
    a.totals[IDX_T_ERR_REC] = stopped && (fl_last & IDX_ERROR) ? tot & REC_MASK : ~0ull;
    a.totals[IDX_T_OVERFLOW] = (tot & REC_MASK) > a.rec_cap || (tot >> REC_BITS) > a.tile_cap ? 1 : 0;
    // set by the write pass, window by window
    a.totals[IDX_T_BAD] = 0;
    a.totals[IDX_T_BADWIN] = 0xffffffffull;
    a.totals[IDX_T_TRIM] = 0;
}

// ---- the write pass: a wave per window puts its tiles and record offsets at its bases ----
__global__ __launch_bounds__(IB) void te_index_write(IdxArgs a) {
    const int lane = threadIdx.x & 63;
    const u32 k = blockIdx.x * IWAVES + (threadIdx.x >> 6);
    if (k >= a.nwin) return;
    // (the loads this wave needs before the copies, issued together)
    u64 *T = a.totals;
    const u64 nwin_chain = T[IDX_T_WINDOWS], ovf = T[IDX_T_OVERFLOW];
    const Part G = ((const Part *)a.parts)[k / SB];
    const u64 agg = a.w_agg[k], lpfx = a.w_pfx[k], wexit = a.w_exit[k], lsb = a.w_sbase[k];
    const u64 eq = a.w_entry[k];
    const long long wprev = a.w_prev[k];
    const u32 wfl = a.w_flags[k];
    if (k >= nwin_chain) return;  // past the chain's end
    constexpr u64 WN = WNB;
    if (lane == 0) {
        // the chain across windows: this window's first record must be where the chain left
        // the nearest earlier window a record starts in; a window without one must be passed
        // over whole (a miss: the caller keeps the host walk's index, which is exact)
        u64 entry;
        const u32 kE = idx_kE(a, entry);
        bool bad = false;
        if (k == kE) {
            bad = eq != entry;
        } else if (k > kE) {
            long long j = G.lastrec > wprev ? G.lastrec : wprev;
            if (j < (long long)kE) j = kE;
            const u64 xj = a.w_exit[j];
            if (eq != IDX_NONE) {
                bad = xj != eq;
            } else {
                const u64 qe = a.base + (u64)(k + 1) * WN;
                bad = xj < (qe < a.len ? qe : a.len) && !(a.w_flags[j] & STOPS);
            }
        }
        if (bad) {
            atomicOr((unsigned long long *)&T[IDX_T_BAD], 1ull);
            atomicMin((unsigned long long *)&T[IDX_T_BADWIN], (unsigned long long)k);
        }
        if (wfl & IDX_TRIM) atomicOr((unsigned long long *)&T[IDX_T_TRIM], 1ull);
    }
    if (ovf) return;
    const u64 ws = a.base + (u64)k * WN;
    const u64 pfx = G.agg + lpfx;
    const u32 nrec = (u32)(agg & REC_MASK), ntile = (u32)(agg >> REC_BITS);
    if (!nrec) return;
    const u64 pbase = pfx & REC_MASK, tbase = pfx >> REC_BITS;
    const u32 rend = (u32)(wexit - ws);  // the window's last record's end
    u64 sb = G.scr + lsb;
    for (u32 t0 = 0; t0 < ntile; t0 += IW) {
        const u32 t = t0 + lane;
        const bool v = t < ntile;
        uint2 me = v ? ((const uint2 *)a.t_tile)[(u64)k * IDX_MAXR + t] : make_uint2(0, 0);
        const u32 nx = t + 1 < ntile ? ((const uint2 *)a.t_tile)[(u64)k * IDX_MAXR + t + 1].x : rend;
        te_tile_t tl;
        tl.span_off = ws + me.x;
        tl.first_pkt = (u32)(pbase + (me.y & 0xffffu));
        tl.npkt = me.y >> 16;
        tl.span_len = nx - me.x;
        tl.flags = 0;
        tl.scratch_off = TE_NO_SCRATCH;
        const u32 g = (u32)(tl.span_off & 15);
        u64 mine = 0;
        if (v && tl.npkt == 1 && !TE_CONTIG_FITS_IN(g, tl.span_len, a.budget)) {
            if (TE_CONTIG_FITS(g, tl.span_len))
                tl.flags = TE_TILE_SOLO;
            else  // a record larger than a tile: its slot in HBM scratch
                mine = ((u64)TE_SLOT_BYTES_OF(g, tl.span_len - 16) + TE_LDS_FRONT + 64 + 255) & ~255ull;
        }
        u64 x = mine;  // inclusive wave scan of the slot bytes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u64 y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (mine) tl.scratch_off = sb + x - mine;
        sb += __shfl(x, 63);
        if (v) a.tiles[tbase + t] = tl;
    }
    for (u32 i = lane; i < nrec; i += IW) a.pkt_rel[pbase + i] = a.t_prel[(u64)k * IDX_MAXR + i];
}
}  // namespace

extern "C" uint32_t te_index_window_bytes(void) { return IW * TE_IDX_S - TE_IDX_OL * TE_IDX_S; }

// count (a wave per window), part (a block per SB windows), scan (one block over the part
// blocks), write (a wave per window): no window waits on another
extern "C" int te_launch_index(const IdxArgs *args, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const IdxArgs a = *args;
    if (a.nwin == 0) return 0;
    const u32 blocks = (a.nwin + IWAVES - 1) / IWAVES;
    hipLaunchKernelGGL((te_index_count<TE_IDX_S, TE_IDX_OL>), dim3(blocks), dim3(IB), 0, st, a);
    hipLaunchKernelGGL(te_index_part, dim3((a.nwin + SB - 1) / SB), dim3(SB), 0, st, a);
    hipLaunchKernelGGL(te_index_scan, dim3(1), dim3(SB), 0, st, a);
    hipLaunchKernelGGL(te_index_write, dim3(blocks), dim3(IB), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
