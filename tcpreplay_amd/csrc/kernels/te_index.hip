// te_index.hip -- the record index on the device (index -> edit -> scan
// -> compaction; 7 hard part 5: chunked speculation).
//
// libpcap reads a capture as a chain of records, each header saying where the next one
// starts (tcprewrite.c:289 pcap_next).  The host walks that chain (te_api.c walk_range);
// here it is found in parallel, speculatively, and checked:
//   * the capture is cut into windows of W bytes, one wave each, and every window into 64
//     sub-windows, one lane each;
//   * a lane guesses its first record start -- the first offset in its sub-window where 8
//     consecutive headers are ones libpcap would accept (the host stretches' test) -- and
//     walks the records that start in its sub-window;
//   * the guesses are checked in order: lane l's first record must be where lane l - 1's
//     walk left off (a lane whose guess was wrong walks again from there), and window k's
//     first record where the chain left the windows before it (in the scan; a wrong guess
//     there sends the batch back to the host walk, which is exact);
//   * lane 0 cuts the window's records into wave-lane tiles as walk_range does (byte budget,
//     64 records, solo and huge records); a tile never spans two windows;
//   * a count pass, a scan over windows (record, tile, byte and scratch bases; the first
//     stop), and a write pass that places every tile and record offset.
// libpcap's ends are kept: an oversize record (caplen > 262144) or a truncated one ends
// the chain; a len > 262144 record ends it with the reference's error (tcprewrite.c:296).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "te_index.h"

namespace {
typedef uint8_t u8;
typedef uint32_t u32;

constexpr int IW = 64;  // lanes (sub-windows) per window

__device__ __forceinline__ u32 rd32u(const u8 *p, bool sw) {  // unaligned
    const u32 v = (u32)p[0] | (u32)p[1] << 8 | (u32)p[2] << 16 | (u32)p[3] << 24;
    return sw ? __builtin_bswap32(v) : v;
}

// 8 consecutive acceptable headers at p (te_api.c chain_plausible)
__device__ bool plausible(const IdxArgs &a, uint64_t p) {
    const u32 lim = a.nsec ? 1000000000u : 1000000u;
    for (int i = 0; i < 8; ++i) {
        if (p + 16 > a.len) return i > 0;
        const u8 *h = a.img + p;
        const u32 frac = rd32u(h + 4, a.sw), cl = rd32u(h + 8, a.sw), pl = rd32u(h + 12, a.sw);
        if (cl > 262144u || pl > 262144u || frac >= lim || p + 16 + cl > a.len) return false;
        p += 16 + (uint64_t)cl;
    }
    return true;
}

// one lane's walk over the records that start in [from, se)
struct LaneWalk {
    uint64_t exit;  // first record start >= se, or where the chain ended
    u32 n;          // records taken
    u32 stop;       // 0 goes on, IDX_STOP oversize, IDX_ERROR len > 262144, IDX_END truncated / no bytes
};

__device__ LaneWalk walk(const IdxArgs &a, uint64_t from, uint64_t se) {
    LaneWalk w{from, 0, 0};
    uint64_t off = from;
    while (off < se) {
        if (off + 16 > a.len) {
            w.stop = IDX_END;
            break;
        }
        const u8 *h = a.img + off;
        const u32 cl = rd32u(h + 8, a.sw), pl = rd32u(h + 12, a.sw);
        if (cl > 262144u) {
            w.stop = IDX_STOP;
            break;
        }
        if (off + 16 + cl > a.len) {
            w.stop = IDX_END;
            break;
        }
        if (pl > 262144u) {
            w.stop = IDX_ERROR;
            break;
        }
        ++w.n;
        off += 16 + (uint64_t)cl;
    }
    w.exit = off;
    return w;
}

template <bool WRITE>
__global__ __launch_bounds__(IW) void te_index_windows(IdxArgs a) {
    extern __shared__ u32 rel[];  // the window's record offsets (from the window start); + the last caplen
    __shared__ u32 base_l[IW + 1];
    const u32 k = blockIdx.x, lane = threadIdx.x;
    if (WRITE && k >= a.totals[IDX_T_WINDOWS]) return;  // past the chain's end
    const uint64_t ws = 24 + (uint64_t)k * a.W;
    const uint64_t we = ws + a.W < a.len ? ws + a.W : a.len;
    const uint64_t sub = a.W / IW;
    auto sub_lo = [&](u32 l) { return ws + l * sub; };
    auto sub_hi = [&](u32 l) { return ws + (l + 1) * sub < we ? ws + (l + 1) * sub : we; };
    // ---- this lane's guess and walk ----
    uint64_t e = IDX_NONE;
    if (k == 0 && lane == 0) {
        e = 24;
    } else {
        for (uint64_t c = sub_lo(lane); c < sub_hi(lane); ++c)
            if (plausible(a, c)) {
                e = c;
                break;
            }
    }
    LaneWalk w = e != IDX_NONE ? walk(a, e, sub_hi(lane)) : LaneWalk{0, 0, 0};
    bool has = e != IDX_NONE;
    // ---- checks in lane order (uniform loop; lane l's values broadcast) ----
    uint64_t cur = IDX_NONE;  // where the chain is (IDX_NONE: not started in this window)
    u32 ended = 0;            // the chain ended in an earlier lane
    for (u32 l = 0; l < IW; ++l) {
        const uint64_t el = __shfl(e, (int)l);
        if (ended) {
            if (lane == l) has = false;
            continue;
        }
        if (cur == IDX_NONE) {  // the window's chain starts at the first guess (checked in the scan)
            if (el != IDX_NONE) {
                cur = __shfl(w.exit, (int)l);
                ended = (u32)__shfl((int)w.stop, (int)l);
            }
            continue;
        }
        if (cur >= sub_hi(l)) {  // a record covers sub-window l: no record starts in it
            if (lane == l) has = false;
            continue;
        }
        if (el != cur && lane == l) {  // a wrong guess: walk again from where the chain is
            e = cur;
            w = walk(a, cur, sub_hi(l));
            has = true;
        }
        cur = __shfl(w.exit, (int)l);
        ended = (u32)__shfl((int)w.stop, (int)l);
    }
    // the window's entry (the first lane in the chain) and how the chain ends here
    uint64_t went = IDX_NONE;
    u32 wstop = 0;
    for (u32 l = 0; l < IW; ++l)
        if (__shfl((int)has, (int)l)) {
            went = __shfl(e, (int)l);
            break;
        }
    for (u32 l = 0; l < IW; ++l) {
        const u32 s = (u32)__shfl((int)(has ? w.stop : 0u), (int)l);
        if (s) {
            wstop = s;
            break;
        }
    }
    // ---- the window's records: counts, positions, offsets in LDS ----
    const u32 n = has ? w.n : 0;
    base_l[lane + 1] = n;
    if (lane == 0) base_l[0] = 0;
    __syncthreads();
    if (lane == 0)
        for (int l = 1; l <= IW; ++l) base_l[l] += base_l[l - 1];
    __syncthreads();
    const u32 nrec = base_l[IW];
    const u32 err_rec = [&] {  // the window-relative index of the record with the len error
        u32 r = 0xffffffffu;
        for (u32 l = 0; l < IW; ++l)
            if (__shfl((int)(has && w.stop == IDX_ERROR), (int)l)) {
                r = base_l[l] + (u32)__shfl((int)n, (int)l);
                break;
            }
        return r;
    }();
    if (has) {
        uint64_t off = e;
        const u32 p = base_l[lane];
        for (u32 i = 0; i < w.n; ++i) {
            rel[p + i] = (u32)(off - ws);
            const u32 cl = rd32u(a.img + off + 8, a.sw);
            if (p + i + 1 == nrec) rel[nrec] = cl;  // the last record's caplen
            off += 16 + (uint64_t)cl;
        }
    }
    __syncthreads();
    // ---- the tile cut (lane 0, as walk_range: budget, max records, solo, huge) ----
    if (lane == 0) {
        u32 ntile = 0, zero = 0;
        uint64_t recbytes = 0, scratch = 0;
        const uint64_t tbase = WRITE ? a.t_base[k] : 0, pbase = WRITE ? a.p_base[k] : 0;
        const uint64_t sbase = WRITE ? a.s_base[k] : 0;
        te_tile_t ct{};
        bool open = false;
        uint64_t t0 = 0;  // the open tile's first record offset
        u32 nxt = nrec ? rel[0] : 0;
        for (u32 i = 0; i < nrec; ++i) {
            const u32 r = nxt;
            nxt = rel[i + 1];  // the next record's offset, or (i + 1 == nrec) the last caplen
            const uint64_t off = ws + r;
            const u32 cl = i + 1 < nrec ? nxt - r - 16 : nxt;
            zero |= cl == 0;
            const u32 g = (u32)(off & 15);
            bool huge = !TE_CONTIG_FITS_IN(g, 16 + cl, a.budget);
            const bool fits = open && TE_CONTIG_FITS_IN(t0 & 15, off + 16 + cl - t0, a.budget);
            const bool solo = huge && TE_CONTIG_FITS(g, 16 + cl);
            if (solo) huge = false;
            if (open && (huge || solo || ct.npkt >= a.max_pkts || !fits)) {
                if (WRITE) a.tiles[tbase + ntile] = ct;
                ++ntile;
                open = false;
            }
            if (!open) {
                ct.span_off = off;
                ct.scratch_off = TE_NO_SCRATCH;
                ct.first_pkt = (u32)(pbase + i);
                ct.npkt = 0;
                ct.span_len = 0;
                ct.flags = 0;
                t0 = off;
                open = true;
            }
            if (WRITE) a.pkt_rel[pbase + i] = (uint16_t)(off - t0);
            ++ct.npkt;
            ct.span_len = (u32)(off + 16 + cl - t0);
            recbytes += 16 + (uint64_t)cl + a.growth;
            if (huge) {  // a record larger than a tile: its slot in HBM scratch
                const u32 slot = TE_SLOT_BYTES_OF(g, cl);
                ct.scratch_off = sbase + scratch;
                scratch += (slot + TE_LDS_FRONT + 64 + 255) & ~255u;
                if (WRITE) a.tiles[tbase + ntile] = ct;
                ++ntile;
                open = false;
            } else if (solo) {
                ct.flags |= TE_TILE_SOLO;
                if (WRITE) a.tiles[tbase + ntile] = ct;
                ++ntile;
                open = false;
            }
        }
        if (open) {
            if (WRITE) a.tiles[tbase + ntile] = ct;
            ++ntile;
        }
        if (!WRITE) {
            a.w_nrec[k] = nrec;
            a.w_ntile[k] = ntile;
            a.w_recbytes[k] = recbytes;
            a.w_scratch[k] = scratch;
            a.w_entry[k] = went;
            a.w_exit[k] = went == IDX_NONE ? IDX_NONE : cur;
            a.w_err[k] = err_rec;
            a.w_flags[k] = wstop | (zero ? IDX_ZERO : 0u);
        }
    }
}

// one block: checks every window's entry against where the chain left the windows before
// it, finds the window where it ends, scans the counts into bases, and writes the totals
__global__ __launch_bounds__(1024) void te_index_scan(IdxArgs a) {
    __shared__ unsigned long long part[4][1024];
    __shared__ unsigned long long bad_at, end_at;
    const u32 t = threadIdx.x, nw = a.nwin;
    if (t == 0) {
        bad_at = ~0ull;
        end_at = ~0ull;
    }
    __syncthreads();
    for (u32 k = t; k < nw; k += 1024) {
        if (a.w_flags[k] & (IDX_STOP | IDX_ERROR | IDX_END)) atomicMin(&end_at, (unsigned long long)k);
        if (k == 0) {
            if (a.w_entry[0] != 24) atomicMin(&bad_at, 0ull);
            continue;
        }
        const uint64_t e = a.w_entry[k];
        if (e == IDX_NONE) continue;  // no record starts here: the next entry is checked instead
        u32 j = k - 1;
        while (j > 0 && a.w_entry[j] == IDX_NONE) --j;  // (records larger than a window only)
        if (a.w_exit[j] != e) atomicMin(&bad_at, (unsigned long long)k);
    }
    __syncthreads();
    const u32 last = end_at == ~0ull ? nw - 1 : (u32)end_at;
    const bool bad = bad_at != ~0ull && bad_at <= last;
    // blocked scan of (records, tiles, bytes, scratch) over windows [0, last]
    const u32 per = (last + 1 + 1023) / 1024, k0 = t * per, k1 = k0 + per < last + 1 ? k0 + per : last + 1;
    unsigned long long s[4] = {0, 0, 0, 0};
    for (u32 k = k0; k < k1; ++k) {
        s[0] += a.w_nrec[k];
        s[1] += a.w_ntile[k];
        s[2] += a.w_recbytes[k];
        s[3] += a.w_scratch[k];
    }
    for (int q = 0; q < 4; ++q) part[q][t] = s[q];
    __syncthreads();
    if (t < 4) {
        unsigned long long run = 0;
        for (u32 i = 0; i < 1024; ++i) {
            const unsigned long long v = part[t][i];
            part[t][i] = run;
            run += v;
        }
        a.totals[IDX_T_RECS + t] = run;
    }
    __syncthreads();
    unsigned long long b[4] = {part[0][t], part[1][t], part[2][t], part[3][t]};
    for (u32 k = k0; k < k1; ++k) {
        a.p_base[k] = b[0];
        a.t_base[k] = b[1];
        a.s_base[k] = b[3];
        b[0] += a.w_nrec[k];
        b[1] += a.w_ntile[k];
        b[2] += a.w_recbytes[k];
        b[3] += a.w_scratch[k];
    }
    if (t == 0) {
        u32 j = last;
        while (j > 0 && a.w_entry[j] == IDX_NONE) --j;
        unsigned long long z = 0;
        for (u32 q = 0; q <= last; ++q) z |= a.w_flags[q] & IDX_ZERO;
        a.totals[IDX_T_BAD] = bad ? 1 : 0;
        a.totals[IDX_T_WINDOWS] = last + 1;
        a.totals[IDX_T_STOP] = end_at == ~0ull ? 0 : (a.w_flags[last] & (IDX_STOP | IDX_ERROR | IDX_END));
        a.totals[IDX_T_END] = a.w_exit[j];
        a.totals[IDX_T_ZERO] = z ? 1 : 0;
        a.totals[IDX_T_ERR_REC] =
            end_at != ~0ull && (a.w_flags[last] & IDX_ERROR) ? a.p_base[last] + a.w_err[last] : ~0ull;
    }
}
}  // namespace

extern "C" int te_launch_index(const IdxArgs *args, int pass, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const IdxArgs a = *args;
    if (a.nwin == 0) return 0;
    const size_t lds = sizeof(u32) * ((size_t)a.W / 16 + 4);
    if (pass == 0)
        hipLaunchKernelGGL(te_index_windows<false>, dim3(a.nwin), dim3(IW), lds, st, a);
    else if (pass == 1)
        hipLaunchKernelGGL(te_index_scan, dim3(1), dim3(1024), 0, st, a);
    else
        hipLaunchKernelGGL(te_index_windows<true>, dim3(a.nwin), dim3(IW), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
