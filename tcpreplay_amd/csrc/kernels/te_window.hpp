// te_window.hpp -- record discovery in one byte window of a pcap image, by one wave:
// the speculative, exactly checked chain search of the device record index (te_index.hip
// count pass), shared with the fused edit (te_wave_tiles' window mode, tcpedit_kernels.hip).
//
// Window k owns the record starts in [ws, we), ws = base + k WN (WN = 64 S - OL S bytes);
// its wave stages [ws - OL S, we + 16) into LDS with coalesced 16-byte loads, the first OL
// lanes' sub-windows establishing the chain entering ws.  A lane guesses the first record
// start in its S-byte sub-window from the zero-byte mask of its dwords (a header has zero
// bytes at +11 and +15 -- caplen, len <= 262144 -- and at +7 for a microsecond capture) and
// walks its records from there; the guesses are reconciled (a lane's guess must be where the
// nearest earlier guessing lane's walk ended: Jacobi rounds, then a serial lane loop).  The
// cross-window chain is checked by the caller (the index's write pass, the fused edit's
// validation kernel): a window's first record must be where the chain left the nearest
// earlier window with a record.  libpcap's ends are kept: an oversize record (caplen >
// 262144) or a truncated one ends the chain; len > 262144, len 0 or caplen 0 ends it with
// safe_pcap_next's exit (src/common/utils.c:131-169).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "te_index.h"

#ifndef TE_WIN_CAND3
#define TE_WIN_CAND3 1  // candidate masks from three dword zero-masks (0: per-byte flag nibbles, A/B)
#endif

namespace tew {
typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

constexpr int IW = 64;          // lanes (sub-windows) per window
constexpr u32 MAXCAP = 262144u;

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
    u32 stop;  // 0 goes on, IDX_STOP oversize, IDX_ERROR the reader's exit, IDX_END truncated / no bytes
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
        if (pl > MAXCAP || pl == 0 || cl == 0) {  // safe_pcap_next exits (utils.c:136-156)
            w.stop = IDX_ERROR;
            break;
        }
        ++w.n;
        off += 16 + (u64)cl;
    }
    w.exit = off;
    return w;
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


// what the discovery leaves: the window's geometry, its records' offsets from ws in rel[0,
// nrec) and the last record's end in rel[nrec], and how the chain enters and leaves it
struct Found {
    u64 ws, we, A0, staged_end;
    u64 went, wexit;  // IDX_NONE: no record starts here
    u32 wstop, nrec;
    bool anytrim;     // a record with len < caplen (safe_pcap_next trims it, utils.c:159-162)
};
// a window's staging: its 16-byte chunks [c0, nch) from A0, in registers (K a lane) until
// stored to LDS -- issued one window ahead by the fused edit, so the loads are in flight
// while it edits the window before
template <int S, int OL, int PRE>
struct Staging {
    static constexpr int W = IW * S, O = OL * S, WN = W - O;
    static constexpr int K = (W + 48 + PRE + 16 * IW - 1) / (16 * IW);
    uint4 v[K];
};

// window k's byte range: [ws, we) owned, staged [lo_stage, staged_end) from A0
template <int S, int OL, int PRE>
__device__ __forceinline__ void window_range(const IdxArgs &a, u32 k, u64 &ws, u64 &we, u64 &A0, u64 &lo_stage,
                                             u64 &staged_end) {
    constexpr int W = IW * S, O = OL * S, WN = W - O;
    ws = a.base + (u64)k * WN;
    we = ws + WN < a.limit ? ws + WN : a.limit;
    A0 = ws - O;  // lane l's sub-window starts at A0 + l S (window 0: none before base)
    lo_stage = k ? A0 : a.base;
    // bytes [lo_stage, staged_end) are in LDS (past a.len: garbage; never more than 16 past it)
    staged_end = PRE == 0 ? we + 16 : (we + 16 + PRE < a.len + 16 ? we + 16 + PRE : (we > a.len ? we : a.len) + 16);
}

// the loads of window k's staging (in flight until stage_store)
template <int S, int OL, int PRE>
__device__ __forceinline__ void stage_load(const IdxArgs &a, u32 k, Staging<S, OL, PRE> &st) {
    u64 ws, we, A0, lo_stage, staged_end;
    window_range<S, OL, PRE>(a, k, ws, we, A0, lo_stage, staged_end);
    const int lane = threadIdx.x & 63;
    const u32 c0 = (u32)((lo_stage - A0) >> 4);
    const u32 nch = (u32)((staged_end - A0 + 15) >> 4);
    const uint4 *g = (const uint4 *)(a.img + A0);
#pragma unroll
    for (int i = 0; i < Staging<S, OL, PRE>::K; ++i) {
        const u32 c = lane + i * IW;
        st.v[i] = (c >= c0 && c < nch) ? g[c] : make_uint4(0, 0, 0, 0);
    }
}

// the staging into LDS (waits for its loads)
template <int S, int OL, int PRE>
__device__ __forceinline__ void stage_store(const IdxArgs &a, u32 k, const Staging<S, OL, PRE> &st, u32 *img) {
    constexpr int W = IW * S;
    u64 ws, we, A0, lo_stage, staged_end;
    window_range<S, OL, PRE>(a, k, ws, we, A0, lo_stage, staged_end);
    const int lane = threadIdx.x & 63;
    const u32 nch = (u32)((staged_end - A0 + 15) >> 4);
#pragma unroll
    for (int i = 0; i < Staging<S, OL, PRE>::K; ++i) {
        const u32 c = lane + i * IW;
        if (c < nch && c < (u32)((W + 48 + PRE) / 16)) *(uint4 *)&img[4 * c] = st.v[i];
    }
}

// img: (W + 48 + PRE) / 4 dwords at least (W = 64 S); rel: 4 S + 1 entries (R: u16 when
// every offset from ws fits, the fused edit's LDS budget).  PRE: bytes
// staged past the window's end + 16 (the fused edit's last record reaching past the window:
// in LDS with the window, no second dependent load for it).  STAGED: the caller has stored
// window k's staging into img already (stage_load / stage_store)
// ts: (diagnostic builds) s_memtime per phase added to ts[0..4]: candidates, walks,
// confirmation, Jacobi rounds, positions -- or null
template <int S, int OL, int PRE = 0, bool STAGED = false, typename R = u32>
__device__ __forceinline__ Found find_window(const IdxArgs &a, u32 *img, R *rel, u32 k,
                                             unsigned long long *ts = nullptr) {
    unsigned long long tl_ = ts ? __builtin_amdgcn_s_memtime() : 0ull;
#define TEW_STAMP(i)                                                    \
    if (ts) {                                                           \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
        ts[i] += now_ - tl_;                                            \
        tl_ = now_;                                                     \
    }
    constexpr int W = IW * S;       // staged sub-window bytes
    constexpr int O = OL * S;       // overlap before the window
    constexpr int WN = W - O;       // bytes a window owns
    static_assert(S % 16 == 0 && S <= 128, "sub-window: whole 16-byte chunks, <= two 64-bit masks");
    const int lane = threadIdx.x & 63;

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
    // bytes [lo_stage, staged_end) are in LDS (past a.len: garbage; never more than 16 past it)
    const u64 staged_end = PRE == 0 ? we + 16 : (we + 16 + PRE < a.len + 16 ? we + 16 + PRE : (we > a.len ? we : a.len) + 16);

    // ---- stage the window: 16-byte chunks, all loads in flight before the LDS stores ----
    if constexpr (!STAGED) {
        const u32 c0 = (u32)((lo_stage - A0) >> 4);
        const u32 nch = (u32)((staged_end - A0 + 15) >> 4);
        const uint4 *g = (const uint4 *)(a.img + A0);
        constexpr int K = (W + 48 + PRE + 16 * IW - 1) / (16 * IW);
        uint4 v[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32 c = lane + i * IW;
            v[i] = (c >= c0 && c < nch) ? g[c] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const u32 c = lane + i * IW;
            if (c < nch && c < (u32)((W + 48 + PRE) / 16)) *(uint4 *)&img[4 * c] = v[i];
        }
    }
    // one wave's LDS accesses are performed in order; the empty asm keeps the compiler from
    // moving a lane's reads of other lanes' stores across them (no block barrier: the
    // block's waves work on their own windows and may have left already)
    asm volatile("" ::: "memory");

    // ---- this lane's guess: the first strong candidate in its sub-window, else the first weak ----
    const u64 lo = A0 + (u64)lane * S, hi_raw = lo + S;
    const u64 hi = hi_raw < we ? hi_raw : we;
    const bool active = lo >= lo_stage && lo < we && (k > kE || (k == kE && lane > laneE));
    u64 e = IDX_NONE;
    if (k == kE && lane == laneE) {
        e = entry;  // the first record is known
    } else if (active) {
        const u32 q0 = (u32)(lo - A0);  // lane S: a multiple of 16
        const bool us = !a.nsec;
        u64 weak = IDX_NONE;
        unsigned long long mh[(S + 63) / 64];
#if TE_WIN_CAND3
        // a header has a zero byte at +11 and +15 (caplen, len <= 262144), and at +7 when the
        // fraction counts microseconds (< 10^6) -- +8, +12 and +4 in a big-endian capture:
        // three bytes 4 apart, so the same byte lane of three consecutive dwords.  Candidate p
        // = 4 D + b - zf for byte lane b of M_D = Z_D & Z_{D+1} & Z_{D+2} (Z: a dword's
        // zero-byte flags), each M_D's four flags gathered into a nibble by one multiply
        // (no per-dword nibble of every byte's flag, no 64-bit realignment of three masks)
        {
            constexpr int ND = S / 4 + 4;  // dwords of bytes [lo, lo + S + 16)
            u32 Z[ND];
#pragma unroll
            for (int c = 0; c < ND / 4; ++c) {
                const uint4 q = *(const uint4 *)&img[(q0 >> 2) + 4 * c];
                Z[4 * c] = zero_bytes(q.x);
                Z[4 * c + 1] = zero_bytes(q.y);
                Z[4 * c + 2] = zero_bytes(q.z);
                Z[4 * c + 3] = zero_bytes(q.w);
            }
            auto gather = [&](auto zfc) {
                constexpr int ZF = decltype(zfc)::value;
#pragma unroll
                for (int h = 0; h < (S + 63) / 64; ++h) mh[h] = 0;
#pragma unroll
                for (int D = 1; D + 2 < ND; ++D) {
                    const u32 M = (us ? Z[D] : 0xffffffffu) & Z[D + 1] & Z[D + 2];
                    const u64 n = (u64)((((M >> 7) & 0x01010101u) * 0x01020408u) >> 24);  // flags of bytes 0..3
                    const int sh = 4 * D - ZF;  // bit of byte lane 0's candidate (unrolled: constants)
                    if (sh < 0) {
                        mh[0] |= n >> (-sh);
                    } else if (sh < S) {
                        mh[sh >> 6] |= n << (sh & 63);
                        if ((sh & 63) > 60 && (sh >> 6) + 1 < (S + 63) / 64) mh[(sh >> 6) + 1] |= n >> (64 - (sh & 63));
                    }
                }
            };
            if (a.sw) gather(std::integral_constant<int, 4>{});
            else gather(std::integral_constant<int, 7>{});
#pragma unroll
            for (int h = 0; h < (S + 63) / 64; ++h) {
                const int span = S - 64 * h;
                if (span < 64) mh[h] &= (1ull << span) - 1ull;
            }
        }
#else
        // zero flags of bytes [lo, lo + S + 16): dword d of the sub-window holds bytes 4d..4d+3
        u64 z[3] = {0, 0, 0};
        // (16-byte LDS reads: the sub-window starts 16-aligned)
#pragma unroll
        for (int c = 0; c < S / 16 + 1; ++c) {
            const uint4 q = *(const uint4 *)&img[(q0 >> 2) + 4 * c];
            const u32 dw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int d = 4 * c + j;
                const u64 f = (u64)nib(zero_bytes(dw[j])) << ((4 * d) & 63);
                z[(4 * d) >> 6] |= f;
            }
        }
        auto bits_at = [&](int h, int sh) -> unsigned long long {  // bits 64h + j (j < 64) of z >> sh
            return sh == 0 ? z[h] : (z[h] >> sh) | (z[h + 1] << (64 - sh));
        };
        // a header has a zero byte at +11 and +15 (caplen, len <= 262144), and at +7 when the
        // fraction counts microseconds (< 10^6) -- the high bytes: +8, +12 and +4 in a
        // big-endian capture
        const int zc = a.sw ? 8 : 11, zl = a.sw ? 12 : 15, zf = a.sw ? 4 : 7;
#pragma unroll
        for (int h = 0; h < (S + 63) / 64; ++h) {
            mh[h] = bits_at(h, zc) & bits_at(h, zl) & (us ? bits_at(h, zf) : ~0ull);
            const int span = S - 64 * h;
            if (span < 64) mh[h] &= (1ull << span) - 1ull;
        }
#endif
        // (one candidate at a time: batching the first four's header reads -- two LDS round
        // trips instead of two each -- ran slower, the lane is issue-bound here)
#pragma unroll
        for (int h = 0; h < (S + 63) / 64; ++h) {
            if (e != IDX_NONE) break;
            unsigned long long m = mh[h];
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const u64 c = lo + 64 * h + j;
                if (c >= hi) break;
                const int st = strength(a, img, A0, staged_end, c);
                if (st == 2) {
                    e = c;
                    break;
                }
                if (st == 1 && weak == IDX_NONE) weak = c;
            }
        }
        if (e == IDX_NONE) e = weak;
    }
    TEW_STAMP(0)
    LaneWalk w = e != IDX_NONE ? walk_lds(a, img, A0, e, hi) : LaneWalk{0, 0, 0};
    bool has = e != IDX_NONE;
    TEW_STAMP(1)

    // ---- where the chain starts: the first guess the next guess confirms (its walk ends
    // exactly there, or at a strong candidate).  A guess that is not a record start jumps by
    // a garbage length, so it is confirmed only when it lands on the chain anyway (and then
    // the chain is right from there on); window 0's known first record needs no
    // confirmation.  Lane sets are ballots: the next guessing lane is a bit search, not a
    // wave scan; offsets travel relative to A0 in 32 bits (a walk ends < 2^20 bytes on) ----
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes < this one
    {
        const unsigned long long hm0 = __ballot(has);
        const unsigned long long after = hm0 & ~below & ~(1ull << lane);
        const int nxt = after ? __builtin_ctzll(after) : 64;
        const u32 ngr = (u32)__shfl((int)(has ? (u32)(e - A0) : 0u), nxt < 64 ? nxt : 0);
        const u64 ng = A0 + ngr;
        // (or its walk ends at a strong candidate inside the window: a wrong guess next to a
        // record start would otherwise hide the record start's confirmation)
        const bool confirmed = has && !w.stop &&
                               ((nxt < 64 && w.exit == ng) ||
                                (w.exit < we && strength(a, img, A0, staged_end, w.exit) == 2));
        const unsigned long long cm = __ballot(confirmed);
        const int start = k == kE ? laneE : (cm ? __builtin_ctzll(cm) : (hm0 ? __builtin_ctzll(hm0) : 64));
        if (lane < start) {
            has = false;
            e = IDX_NONE;
        }
    }
    TEW_STAMP(2)

    // ---- the exact chain: the chain's first guess is trusted (the overlap lanes' chain, or window 0's
    // known first record); after it, lane l's first record must be where the nearest earlier
    // guessing lane's walk ended (P), and no lane the chain passes over may keep a guess.
    // Jacobi rounds, each fixing at least the first inconsistent lane, until every lane agrees
    // (in practice one or two); the serial lane loop after 8 rounds.  The nearest earlier
    // guessing lane is a bit search on the ballot; its exit and stop come in one shuffle ----
    bool settled = false;
    for (int round = 0; round < 8; ++round) {
        const unsigned long long hb = __ballot(has) & below;
        const int prev = hb ? 63 - __builtin_clzll(hb) : -1;
        const u32 xs = (u32)__shfl((int)((((u32)(w.exit - A0)) << 3) | w.stop), prev < 0 ? 0 : prev);
        const u64 P = A0 + (xs >> 3);
        const u32 pstop = xs & 7u;
        bool change = false;
        if (prev >= 0 && active) {
            if (pstop) {  // the chain ended before this lane
                change = has;
                has = false;
            } else if (P < lo) {  // (an earlier lane without a guess takes it first)
            } else if (P < hi) {  // the chain enters this sub-window at P
                if (!has || e != P) {
                    e = P;
                    w = walk_lds(a, img, A0, P, hi);
                    has = true;
                    change = true;
                }
            } else if (has) {  // the chain passes over it
                has = false;
                change = true;
            }
        }
        if (!__ballot(change)) {
            settled = true;
            break;
        }
    }
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
                w = walk_lds(a, img, A0, cur, lh);
                has = true;
            }
            cur = __shfl(w.exit, (int)l);
            ended = (u32)__shfl((int)w.stop, (int)l);
        }
    }
    TEW_STAMP(3)
    // only the window's own lanes' records count (the overlap's are window k - 1's)
    if (lane < OL) has = false;
    // the window's entry, exit and how the chain ends here (wave-uniform lanes: readlane)
    const unsigned long long hm = __ballot(has);
    const int fl = hm ? __builtin_ctzll(hm) : 0, ll = hm ? 63 - __builtin_clzll(hm) : 0;
    const u64 went = hm ? A0 + (u32)__builtin_amdgcn_readlane((int)(u32)(e - A0), fl) : IDX_NONE;
    const u32 xl = (u32)__builtin_amdgcn_readlane((int)((((u32)(w.exit - A0)) << 3) | w.stop), ll);
    const u64 wexit = hm ? A0 + (xl >> 3) : IDX_NONE;
    const u32 wstop = hm ? (xl & 7u) : 0u;
    // ---- the window's records: positions, offsets into LDS.  A lane takes at most S / 16
    // records (< 8): its count's three bits are three ballots, its position their popcounts
    // below it ----
    static_assert(S / 16 < 16, "a lane's record count fits four bits");
    const u32 n = has ? w.n : 0;
    const unsigned long long n0 = __ballot(n & 1u), n1 = __ballot(n & 2u), n2 = __ballot(n & 4u),
                             n3 = S / 16 >= 8 ? __ballot(n & 8u) : 0ull;
    const u32 pos = (u32)(__builtin_popcountll(n0 & below) + 2 * __builtin_popcountll(n1 & below) +
                          4 * __builtin_popcountll(n2 & below) + 8 * __builtin_popcountll(n3 & below));
    const u32 nrec = (u32)(__builtin_popcountll(n0) + 2 * __builtin_popcountll(n1) + 4 * __builtin_popcountll(n2) +
                           8 * __builtin_popcountll(n3));
    bool zero = false;
    if (has) {
        u64 off = e;
        for (u32 i = 0; i < w.n; ++i) {
            rel[pos + i] = (R)(off - ws);
            const u32 cl = sw32(lds_u32(img, (u32)(off - A0) + 8), a.sw),
                      pl = sw32(lds_u32(img, (u32)(off - A0) + 12), a.sw);
            zero |= pl < cl;  // safe_pcap_next trims it: the exact path places it by scan
            off += 16 + (u64)cl;
            if (pos + i + 1 == nrec) rel[nrec] = (R)(off - ws);  // the last record's end
        }
    }
    const bool anytrim = __ballot(zero) != 0;
    asm volatile("" ::: "memory");
    TEW_STAMP(4)
#undef TEW_STAMP
    return Found{ws, we, A0, staged_end, went, wexit, wstop, nrec, anytrim};
}
}  // namespace tew
