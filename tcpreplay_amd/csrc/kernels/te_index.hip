// te_index.hip -- the record index on the device (index -> edit -> scan
// -> compaction; 7 hard part 5: chunked speculation).
//
// libpcap reads a capture as a chain of records, each header saying where the next one
// starts (tcprewrite.c:289 pcap_next).  The host walks that chain (te_api.c walk_range);
// here it is found in parallel, speculatively, and checked exactly, in ONE pass over the
// bytes:
//   * the capture is cut into windows of W = 64 S bytes, one wave each (windows taken in
//     order from an atomic ticket), and every window into 64 sub-windows of S bytes, one
//     lane each.  The wave stages its window (+ 16 bytes) into LDS with coalesced 16-byte
//     loads; every later read is an LDS read;
//   * a lane guesses the first record start in its sub-window: a record header has a zero
//     byte at +11 (caplen <= 262144) and +15 (len <= 262144), and at +7 for a microsecond
//     capture (fraction < 10^6), so the lane builds the sub-window's zero-byte mask from
//     its dwords and tests only the offsets the mask allows -- the header's ranges, and
//     the next header's when it is staged;
//   * each lane walks the records that start in its sub-window from its guess; the guesses
//     are then checked exactly: a lane's guess must be where the nearest earlier lane's
//     walk ended, and no sub-window the chain enters may be without a guess (ballots; a
//     miss re-walks the window lane by lane from where the chain is);
//   * the window's records are cut into wave-lane tiles as walk_range cuts them (byte
//     budget, 64 records, solo and huge records) by a ballot per tile; a tile never spans
//     two windows;
//   * a decoupled look-back over windows (records | tiles in one 64-bit granule) gives the
//     window's first record and tile numbers, and the wave writes its tiles and record
//     offsets in place;
//   * once its look-back has seen every earlier window's granule, a window checks its first
//     record against where the chain left the nearest earlier window with a record (window
//     kE starts at the known first record) and reports a miss as the first bad window;
//     te_index_finish (one lane, the next launch) compares the first bad window with the
//     first stop, finds where the chain ends and writes the totals.  A guess that was wrong
//     across windows sets IDX_T_BAD: the caller keeps the host walk's index, which is exact.
//     (A serial finishing loop over every window cost ~50 ns a window: 0.84 ms on C2.)
// libpcap's ends are kept: an oversize record (caplen > 262144) or a truncated one ends
// the chain; a len > 262144 record ends it with the reference's error (tcprewrite.c:296).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "te_index.h"

// TE_IDX_STAMPS builds (diagnostics only): s_memtime per phase of a few windows, printed
#if TE_IDX_STAMPS
#define IX_STAMP(i) do { __builtin_amdgcn_sched_barrier(0); ix_t[i] = __builtin_amdgcn_s_memtime(); \
                         __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define IX_STAMP(i)
#endif
namespace {
typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

constexpr int IW = 64;                       // lanes (sub-windows) per window
constexpr int IB = 256;                      // threads per block: 4 windows in flight
constexpr int IWAVES = IB / IW;
constexpr u32 MAXCAP = 262144u;
constexpr u64 F_AGG = 1ull << 62, F_PFX = 2ull << 62, VMASK = (1ull << 62) - 1;
constexpr int REC_BITS = 36;                 // granule value: records | tiles << 36
constexpr u64 REC_MASK = (1ull << REC_BITS) - 1;

// one wave's LDS: the staged window, its record offsets, per-record tile starts, tile starts
template <int S>
struct WinLds {
    static constexpr int W = IW * S;
    static constexpr int MAXR = W / 16;      // records starting in a window, at most
    u32 img[(W + 48) / 4];                   // bytes [A0, A0 + W + 48): A0 = window start & ~15
    u32 rel[MAXR + 1];                       // record offset from the window start (+ end of the last)
    u16 tsi[MAXR];                           // the record's tile's first record
    u16 tst[MAXR + 1];                       // tile start records (+ nrec)
    u64 pfx;                                 // the window's exclusive (records | tiles) prefix
};

__device__ __forceinline__ u32 lds_u32(const u32 *img, u32 p) {  // unaligned LDS dword
    const u32 a = img[p >> 2], b = img[(p >> 2) + 1];
    return __builtin_amdgcn_alignbyte(b, a, p & 3u);
}
__device__ __forceinline__ u32 sw32(u32 v, bool sw) { return sw ? __builtin_bswap32(v) : v; }
// a byte's zero mask over a dword: bit 8i+7 set iff byte i == 0 (exact)
__device__ __forceinline__ u32 zero_bytes(u32 x) {
    const u32 y = (x & 0x7f7f7f7fu) + 0x7f7f7f7fu;
    return ~(y | x | 0x7f7f7f7fu);
}
__device__ __forceinline__ u32 nib(u32 z) {  // 4 zero flags of a dword -> 4 bits
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// one lane's walk over the records that start in [from, se), headers from LDS
struct LaneWalk {
    u64 exit;  // first record start >= se, or where the chain ended
    u32 n;     // records taken
    u32 stop;  // 0 goes on, IDX_STOP oversize, IDX_ERROR len > 262144, IDX_END truncated / no bytes
};
__device__ __forceinline__ LaneWalk walk_lds(const IdxArgs &a, const u32 *img, u64 A0, u64 from, u64 se) {
    LaneWalk w{from, 0, 0};
    u64 off = from;
    while (off < se) {
        if (off + 16 > a.len) {
            w.stop = IDX_END;
            break;
        }
        const u32 p = (u32)(off - A0);
        const u32 cl = sw32(lds_u32(img, p + 8), a.sw), pl = sw32(lds_u32(img, p + 12), a.sw);
        if (cl > MAXCAP) {
            w.stop = IDX_STOP;
            break;
        }
        if (off + 16 + cl > a.len) {
            w.stop = IDX_END;
            break;
        }
        if (pl > MAXCAP) {
            w.stop = IDX_ERROR;
            break;
        }
        ++w.n;
        off += 16 + (u64)cl;
    }
    w.exit = off;
    return w;
}

// decoupled look-back over windows, one wave (tcpedit_kernels.hip's, for 64-bit packed
// granules {flag:2 | value:62}, relaxed agent-scope atomics: the value is the hand-off)
__device__ u64 lookback(u64 *state, u32 t, u64 agg, u32 *timeouts) {
    const int lane = threadIdx.x & 63;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(&state[0], F_PFX | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&state[t], F_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    int64_t j = (int64_t)t - 1;
    unsigned spins = 0;
    while (j >= 0) {
        const int64_t idx = j - lane;
        u64 g = F_PFX;
        if (idx >= 0) g = __hip_atomic_load(&state[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 f = g & ~VMASK;
        const u64 pm = __ballot(f == F_PFX), zm = __ballot(f == 0);
        const int first_p = pm ? __builtin_ctzll(pm) : 64;
        const int first_z = zm ? __builtin_ctzll(zm) : 64;
        const int take = first_z < first_p ? first_z : (first_p < 64 ? first_p + 1 : 64);
        u64 v = lane < take ? (g & VMASK) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (first_p < first_z) break;
        j -= take;
        if (first_z < 64) {
            if (++spins > (1u << 24)) {  // bounded spin: report and give up
                if (lane == 0) atomicAdd(timeouts, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0)
        __hip_atomic_store(&state[t], F_PFX | ((excl + agg) & VMASK), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// a candidate's strength: 0 no header here, 1 a header whose successor is not staged (or
// past the image), 2 a header followed by a staged acceptable one (or ending the image)
__device__ __forceinline__ int strength(const IdxArgs &a, const u32 *img, u64 A0, u64 staged_end, u64 p) {
    const u32 lim = a.nsec ? 1000000000u : 1000000u;
    if (p + 16 > a.len) return 0;
    u32 q = (u32)(p - A0);
    u32 frac = sw32(lds_u32(img, q + 4), a.sw), cl = sw32(lds_u32(img, q + 8), a.sw), pl = sw32(lds_u32(img, q + 12), a.sw);
    if (cl > MAXCAP || pl > MAXCAP || frac >= lim || p + 16 + cl > a.len) return 0;
    p += 16 + (u64)cl;
    if (p == a.len) return 2;
    if (p + 16 > a.len || p + 16 > staged_end) return 1;
    q = (u32)(p - A0);
    frac = sw32(lds_u32(img, q + 4), a.sw), cl = sw32(lds_u32(img, q + 8), a.sw), pl = sw32(lds_u32(img, q + 12), a.sw);
    return (cl > MAXCAP || pl > MAXCAP || frac >= lim || p + 16 + cl > a.len) ? 0 : 2;
}

// Window geometry: window k owns the record starts in [ws, we), ws = base + k WN.  Its wave
// stages [ws - O, we + 16): the O = OL S bytes before the window are the first OL lanes'
// sub-windows, whose only job is to establish the chain entering ws (a guess there that is
// not a record start is corrected as the chain runs on, or leaves the window before ws).
template <int S, int OL>
__global__ __launch_bounds__(IB) void te_index_windows(IdxArgs a) {
    constexpr int W = IW * S;       // staged sub-window bytes
    constexpr int O = OL * S;       // overlap before the window
    constexpr int WN = W - O;       // bytes a window owns
    static_assert(S % 16 == 0 && S <= 128, "sub-window: whole 16-byte chunks, <= two 64-bit masks");
    __shared__ WinLds<S> L[IWAVES];
    __shared__ u32 blk_ticket;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WinLds<S> &M = L[wv];
    // one ticket a block (its waves take consecutive windows): windows are numbered in the
    // order blocks start, so a window's look-back only waits on windows already running
    if (threadIdx.x == 0) blk_ticket = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const u32 k = blk_ticket * IWAVES + (u32)wv;
    if (k >= a.nwin) return;
#if TE_IDX_STAMPS
    unsigned long long ix_t[10] = {};
    int ix_rounds = 0;
#endif
    IX_STAMP(0);
    // the first record: known to the host (a.entry), or where the previous pipeline chunk's
    // chain ended (read on the device: that chunk's index ran before this one on the stream)
    const u64 entry = a.entry_ptr ? *(const volatile u64 *)a.entry_ptr - a.entry_sub : a.entry;
    const u64 base = a.base;         // the window grid (16-aligned, <= entry)
    const u64 limit = a.limit;       // records starting here or later are not this image's
    const u32 kE = (u32)((entry - base) / WN);                     // the window of the first record
    const int laneE = OL + (int)(((entry - base) % WN) / S);       // ... and its lane
    const u64 ws = base + (u64)k * WN;
    const u64 we = ws + WN < limit ? ws + WN : limit;
    const u64 A0 = ws - O;          // lane l's sub-window starts at A0 + l S (window 0: none before base)
    const u64 lo_stage = k ? A0 : base;
    const u64 staged_end = we + 16;  // bytes [lo_stage, staged_end) are in LDS (past a.len: garbage)

    // ---- stage the window: 16-byte chunks, all loads in flight before the LDS stores ----
    {
        const u32 c0 = (u32)((lo_stage - A0) >> 4);
        const u32 nch = (u32)((staged_end - A0 + 15) >> 4);
        const uint4 *g = (const uint4 *)(a.img + A0);
        constexpr int K = (W + 48 + 16 * IW - 1) / (16 * IW);
        uint4 v[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32 c = lane + i * IW;
            v[i] = (c >= c0 && c < nch) ? g[c] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32 c = lane + i * IW;
            if (c < nch && c < (u32)((W + 48) / 16)) *(uint4 *)&M.img[4 * c] = v[i];
        }
    }
    // one wave's LDS accesses are performed in order; the empty asm keeps the compiler from
    // moving a lane's reads of other lanes' stores across them (no block barrier: the
    // block's waves work on their own windows and may have left already)
    asm volatile("" ::: "memory");
    IX_STAMP(1);

    // ---- this lane's guess: the first strong candidate in its sub-window, else the first weak ----
    const u64 lo = A0 + (u64)lane * S, hi_raw = lo + S;
    const u64 hi = hi_raw < we ? hi_raw : we;
    const bool active = lo >= lo_stage && lo < we && (k > kE || (k == kE && lane > laneE));
    u64 e = IDX_NONE;
    if (k == kE && lane == laneE) {
        e = entry;  // the first record is known
    } else if (active) {
        // zero flags of bytes [lo, lo + S + 16): dword d of the sub-window holds bytes 4d..4d+3
        const u32 q0 = (u32)(lo - A0);  // lane S: a multiple of 16
        u64 z[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < S / 4 + 4; ++d) {
            const u64 f = (u64)nib(zero_bytes(M.img[(q0 >> 2) + d])) << ((4 * d) & 63);
            z[(4 * d) >> 6] |= f;
        }
        auto bits_at = [&](int h, int sh) -> unsigned long long {  // bits 64h + j (j < 64) of z >> sh
            return sh == 0 ? z[h] : (z[h] >> sh) | (z[h + 1] << (64 - sh));
        };
        // a header has a zero byte at +11 and +15 (caplen, len <= 262144), and at +7 when the
        // fraction counts microseconds (< 10^6) -- the high bytes: +8, +12 and +4 in a
        // big-endian capture
        const bool us = !a.nsec;
        const int zc = a.sw ? 8 : 11, zl = a.sw ? 12 : 15, zf = a.sw ? 4 : 7;
        u64 weak = IDX_NONE;
#pragma unroll
        for (int h = 0; h < (S + 63) / 64; ++h) {
            if (e != IDX_NONE) break;
            unsigned long long m = bits_at(h, zc) & bits_at(h, zl) & (us ? bits_at(h, zf) : ~0ull);
            const int span = S - 64 * h;
            if (span < 64) m &= (1ull << span) - 1ull;
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const u64 c = lo + 64 * h + j;
                if (c >= hi) break;
                const int st = strength(a, M.img, A0, staged_end, c);
                if (st == 2) {
                    e = c;
                    break;
                }
                if (st == 1 && weak == IDX_NONE) weak = c;
            }
        }
        if (e == IDX_NONE) e = weak;
    }
    LaneWalk w = e != IDX_NONE ? walk_lds(a, M.img, A0, e, hi) : LaneWalk{0, 0, 0};
    bool has = e != IDX_NONE;
    IX_STAMP(2);

    // ---- where the chain starts: the first guess the next guess confirms (its walk ends
    // exactly there, or at a strong candidate).  A guess that is not a record start jumps by a garbage length, so it is
    // confirmed only when it lands on the chain anyway (and then the chain is right from
    // there on); window 0's known first record needs no confirmation ----
    {
        int nsrc = has ? lane : 64;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_down(nsrc, o, 64);
            if (lane + o < 64 && y < nsrc) nsrc = y;
        }
        int nxt = __shfl_down(nsrc, 1, 64);
        if (lane == 63) nxt = 64;
        const u64 ng = __shfl(e, nxt < 64 ? nxt : 0);
        // (or its walk ends at a strong candidate inside the window: a wrong guess next to a
        // record start would otherwise hide the record start's confirmation)
        const bool confirmed = has && !w.stop &&
                               ((nxt < 64 && w.exit == ng) ||
                                (w.exit < we && strength(a, M.img, A0, staged_end, w.exit) == 2));
        const u64 cm = __ballot(confirmed), hm0 = __ballot(has);
        const int start = k == kE ? laneE : (cm ? __builtin_ctzll(cm) : (hm0 ? __builtin_ctzll(hm0) : 64));
        if (lane < start) {
            has = false;
            e = IDX_NONE;
        }
    }

    // ---- the exact chain: the chain's first guess is trusted (the overlap lanes' chain, or window 0's
    // known first record); after it, lane l's first record must be where the nearest earlier
    // guessing lane's walk ended (P), and no lane the chain passes over may keep a guess.
    // Jacobi rounds, each fixing at least the first inconsistent lane, until every lane agrees
    // (in practice one or two); the serial lane loop after 8 rounds ----
    bool settled = false;
    for (int round = 0; round < 8; ++round) {
        int src = has ? lane : -1;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(src, o, 64);
            if (lane >= o && y > src) src = y;
        }
        int prev = __shfl_up(src, 1, 64);
        if (lane == 0) prev = -1;
        const u64 P = __shfl(w.exit, prev < 0 ? 0 : prev);
        const u32 pstop = (u32)__shfl((int)w.stop, prev < 0 ? 0 : prev);
        bool change = false;
        if (prev >= 0 && active) {
            if (pstop) {  // the chain ended before this lane
                change = has;
                has = false;
            } else if (P < lo) {  // (an earlier lane without a guess takes it first)
            } else if (P < hi) {  // the chain enters this sub-window at P
                if (!has || e != P) {
                    e = P;
                    w = walk_lds(a, M.img, A0, P, hi);
                    has = true;
                    change = true;
                }
            } else if (has) {  // the chain passes over it
                has = false;
                change = true;
            }
        }
#if TE_IDX_STAMPS
        ix_rounds = round + 1;
#endif
        if (!__ballot(change)) {
            settled = true;
            break;
        }
    }
    IX_STAMP(3);
    if (!settled) {  // the serial lane loop (exact)
        u64 cur = IDX_NONE;
        u32 ended = 0;
        for (u32 l = 0; l < IW; ++l) {
            const u64 ll = A0 + (u64)l * S, lh = ll + S < we ? ll + S : we;
            const bool act = ll >= lo_stage && ll < we && (k > kE || (k == kE && (int)l >= laneE));
            const bool hl = __shfl((int)has, (int)l) != 0;
            if (!act || ended) {
                if (lane == (int)l) has = false;
                continue;
            }
            if (cur == IDX_NONE) {
                if (hl) {
                    cur = __shfl(w.exit, (int)l);
                    ended = (u32)__shfl((int)w.stop, (int)l);
                }
                continue;
            }
            if (cur >= lh) {
                if (lane == (int)l) has = false;
                continue;
            }
            if (lane == (int)l && (!has || e != cur)) {
                e = cur;
                w = walk_lds(a, M.img, A0, cur, lh);
                has = true;
            }
            cur = __shfl(w.exit, (int)l);
            ended = (u32)__shfl((int)w.stop, (int)l);
        }
    }
    IX_STAMP(4);
    // only the window's own lanes' records count (the overlap's are window k - 1's)
    if (lane < OL) has = false;
    // the window's entry, exit and how the chain ends here
    const u64 hm = __ballot(has);
    const int fl = hm ? __builtin_ctzll(hm) : 0, ll = hm ? 63 - __builtin_clzll(hm) : 0;
    const u64 went = hm ? __shfl(e, fl) : IDX_NONE;
    const u64 wexit = hm ? __shfl(w.exit, ll) : IDX_NONE;
    const u32 wstop = hm ? (u32)__shfl((int)w.stop, ll) : 0u;
    // ---- the window's records: positions (wave scan), offsets into LDS ----
    const u32 n = has ? w.n : 0;
    u32 pos = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(pos, o, 64);
        if (lane >= o) pos += y;
    }
    const u32 nrec = __shfl(pos, 63);
    pos -= n;
    bool zero = false;
    if (has) {
        u64 off = e;
        for (u32 i = 0; i < w.n; ++i) {
            M.rel[pos + i] = (u32)(off - ws);
            const u32 cl = sw32(lds_u32(M.img, (u32)(off - A0) + 8), a.sw);
            zero |= cl == 0;
            off += 16 + (u64)cl;
            if (pos + i + 1 == nrec) M.rel[nrec] = (u32)(off - ws);  // the last record's end
        }
    }
    const bool anyzero = __ballot(zero) != 0;
    asm volatile("" ::: "memory");

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
    IX_STAMP(5);

    // ---- the window's record and tile numbers ----
    const u64 agg = (u64)nrec | ((u64)ntile << REC_BITS);
    // publish where the chain enters and leaves this window before the aggregate: a later
    // window reads them once its look-back has seen this window's granule (release here,
    // acquire there)
    if (lane == 0) {
        a.w_entry[k] = went;
        a.w_exit[k] = wexit;
        a.w_flags[k] = wstop;
        __threadfence();
    }
    IX_STAMP(6);
    const u64 excl = lookback(a.state, k, agg, a.timeouts);
    const u64 pbase = excl & REC_MASK, tbase = excl >> REC_BITS;
    IX_STAMP(7);
    if (lane == 0) {
        a.w_pfx[k] = excl + agg;
        if (wstop == IDX_ERROR) a.w_err[k] = pbase + nrec;  // the record the chain stopped at
        // (zeroed words: max of ~k = the first such window)
        if (wstop) atomicMax(a.stop_win_c, ~k);
        if (anyzero) atomicMax(a.zero_win_c, ~k);
        // the chain across windows, checked here: every earlier window has published (the
        // look-back saw their granules).  This window's first record must be where the chain
        // left the nearest earlier window a record starts in; a window without one must be
        // passed over whole.  Only windows up to the chain's end matter: the finishing pass
        // compares the first bad window with the first stop.
        __threadfence();
        bool bad = false;
        if (k == kE) {
            bad = went != entry;
        } else if (k > kE) {
            u32 j = k - 1;
            while (j > kE && ((volatile u64 *)a.w_entry)[j] == IDX_NONE) --j;
            const u64 xj = ((volatile u64 *)a.w_exit)[j];
            if (went != IDX_NONE) {
                bad = xj != went;
            } else {
                const u64 qe = base + (u64)(k + 1) * WN;
                bad = xj < (qe < a.len ? qe : a.len) &&
                      !(((volatile u32 *)a.w_flags)[j] & (IDX_STOP | IDX_ERROR | IDX_END));
            }
        }
        if (bad) atomicMax(a.bad_win_c, ~k);
    }

    // ---- tiles and record offsets in place ----
    bool ovf = false;
    for (u32 t = lane; t < ntile; t += IW) {
        const u32 s0 = M.tst[t], s1 = M.tst[t + 1];
        te_tile_t tl;
        tl.span_off = ws + M.rel[s0];
        tl.first_pkt = (u32)(pbase + s0);
        tl.npkt = s1 - s0;
        tl.span_len = (u32)(M.rel[s1] - M.rel[s0]);
        tl.flags = 0;
        tl.scratch_off = TE_NO_SCRATCH;
        const u32 g = (u32)(tl.span_off & 15);
        if (tl.npkt == 1 && !TE_CONTIG_FITS_IN(g, tl.span_len, a.budget)) {
            if (TE_CONTIG_FITS(g, tl.span_len)) {
                tl.flags = TE_TILE_SOLO;
            } else {  // a record larger than a tile: its slot in HBM scratch
                const u32 slot = TE_SLOT_BYTES_OF(g, tl.span_len - 16);
                const u64 sb = (slot + TE_LDS_FRONT + 64 + 255) & ~255ull;
                tl.scratch_off = atomicAdd((unsigned long long *)a.scratch_ctr, (unsigned long long)sb);
            }
        }
        if (tbase + t < a.tile_cap) a.tiles[tbase + t] = tl;
        else ovf = true;
    }
    for (u32 i = lane; i < nrec; i += IW) {
        if (pbase + i < a.rec_cap) a.pkt_rel[pbase + i] = (u16)(M.rel[i] - M.rel[M.tsi[i]]);
        else ovf = true;
    }
    // (a window past the chain's end counts records that are not -- it may overflow: only
    // the windows up to the end are looked at)
    if (__ballot(ovf) && lane == 0) atomicMax(a.ovf_win_c, ~k);
#if TE_IDX_STAMPS
    IX_STAMP(8);
    if (lane == 0 && (k < 3 || k % 4096 == 0 || k + 1 == a.nwin))
        printf("IX win %u/%u settled %d rounds %d nrec %u ntile %u | stage %llu guess %llu jacobi %llu serial %llu "
               "pos %llu cut %llu lookback %llu write %llu\n", k, a.nwin, (int)settled, ix_rounds, nrec, ntile,
               ix_t[1] - ix_t[0], ix_t[2] - ix_t[1], ix_t[3] - ix_t[2], ix_t[4] - ix_t[3], ix_t[5] - ix_t[4],
               ix_t[6] - ix_t[5], ix_t[7] - ix_t[6], ix_t[8] - ix_t[7]);
#endif
}

// the totals, after every window is done (one wave, the next kernel on the stream)
__global__ __launch_bounds__(64) void te_index_finish(IdxArgs a) {
    const int lane = threadIdx.x;
    if (lane != 0) return;
    const u64 entry = a.entry_ptr ? *(const volatile u64 *)a.entry_ptr - a.entry_sub : a.entry;
    constexpr int WN = IW * TE_IDX_S - TE_IDX_OL * TE_IDX_S;
    const u32 kE = (u32)((entry - a.base) / WN);
    const u32 stop_c = *a.stop_win_c, bad_c = *a.bad_win_c, zero_c = *a.zero_win_c, ovf_c = *a.ovf_win_c;
    const u32 last = stop_c ? ~stop_c : a.nwin - 1;  // windows past the chain's end do not count
    const bool bad = bad_c && ~bad_c <= last;
    u32 j = last;
    while (j > kE && a.w_entry[j] == IDX_NONE) --j;
    const u64 tot = a.w_pfx[last];
    const u32 fl = a.w_flags[last];
    const bool stopped = stop_c != 0;
    a.totals[IDX_T_RECS] = tot & REC_MASK;
    a.totals[IDX_T_TILES] = tot >> REC_BITS;
    a.totals[IDX_T_SCRATCH] = *a.scratch_ctr;
    a.totals[IDX_T_BAD] = bad || *a.timeouts ? 1 : 0;
    a.totals[IDX_T_WINDOWS] = last + 1;
    a.totals[IDX_T_STOP] = stopped ? (fl & (IDX_STOP | IDX_ERROR | IDX_END)) : 0;
    const u64 end = a.w_exit[j];
    a.totals[IDX_T_END] = end == IDX_NONE ? entry : end;
    a.totals[IDX_T_BYTES] = (a.totals[IDX_T_END] - entry) + (u64)a.growth * (tot & REC_MASK);
    a.totals[IDX_T_ZERO] = zero_c && ~zero_c <= last ? 1 : 0;
    a.totals[IDX_T_ERR_REC] = stopped && (fl & IDX_ERROR) ? a.w_err[last] : ~0ull;
    a.totals[IDX_T_OVERFLOW] = ovf_c && ~ovf_c <= last ? 1 : 0;
    a.totals[IDX_T_BADWIN] = bad ? ~bad_c : 0xffffffffu;
}
}  // namespace

extern "C" uint32_t te_index_window_bytes(void) { return IW * TE_IDX_S - TE_IDX_OL * TE_IDX_S; }

// the workspace words the pass needs zeroed (state granules, ticket, done, stop, counters)
extern "C" int te_launch_index(const IdxArgs *args, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const IdxArgs a = *args;
    if (a.nwin == 0) return 0;
    const u32 blocks = (a.nwin + IWAVES - 1) / IWAVES;
    hipLaunchKernelGGL((te_index_windows<TE_IDX_S, TE_IDX_OL>), dim3(blocks), dim3(IB), 0, st, a);
    hipLaunchKernelGGL(te_index_finish, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
