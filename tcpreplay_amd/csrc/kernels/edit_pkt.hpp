// edit_pkt.hpp -- per-packet tcpedit logic for gfx950, one packet per lane.
//
// Restates the reference's per-packet path (src/tcpedit/tcpedit.c:46-366 and
// everything it calls, DLT_EN10MB in and out) over a packet "slot": the packet's
// 16-byte pcap record header followed by its bytes, staged in LDS by the tile
// kernel (or in an HBM scratch slot for packets larger than a tile), with
//   * >= 4 bytes of headroom before the record header, so a VLAN push shifts the
//     (short) L2 head left instead of memmove-ing the whole payload right, and
//   * TE_TAIL zeroed bytes after the payload, the only bytes past caplen that the
//     reference may legitimately touch without depending on an earlier packet.
// Anything the reference would READ past caplen (its static buffer's stale bytes,
// SURVEY Appendix B Q8) is detected and flagged TE_ST_UNSUPPORTED instead.
//
// Byte order: like the reference on x86, multi-byte fields are loaded in host
// (little-endian) order and all checksum arithmetic runs on those LE values.
#pragma once
#ifdef TE_HOST_EMU  // host build of the same logic, for debugging harnesses only
#include <stdint.h>
#define __device__
#define __forceinline__ inline
#else
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>
#include "te_dev_cfg.h"
#include "te_kernels.h"

namespace te {

constexpr int TE_TAIL = TE_TAIL_BYTES;    // zeroed bytes materialised after each packet
constexpr uint32_t MAX_SNAPLEN = 262144;  // defines.h.in:177
constexpr uint32_t MAXPACKET = MAX_SNAPLEN + 22;

constexpr int RC_SOFT = -2, RC_ERROR = -1, RC_OK = 0, RC_WARN = 1;  // tcpedit_types.h:31-34

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;

#define DI __device__ __forceinline__

DI u16 bswap16(u16 v) { return (u16)((v >> 8) | (v << 8)); }
DI u32 bswap32(u32 v) { return __builtin_bswap32(v); }
DI u16 ld16(const u8 *p) { return (u16)(p[0] | (p[1] << 8)); }
DI u32 ld32(const u8 *p) { return (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24); }
DI void st16(u8 *p, u16 v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); }
DI void st32(u8 *p, u32 v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); p[2] = (u8)(v >> 16); p[3] = (u8)(v >> 24); }
DI u16 be16(const u8 *p) { return (u16)((p[0] << 8) | p[1]); }  // ntohs(ld16)
DI u32 be32(const u8 *p) { return bswap32(ld32(p)); }

// ---------------------------------------------------------------------------
// Per-packet context: what the slot holds and what the reference's
// tcpeditdlt_t / en10mb_extra_t decode state carries for this packet.
// ---------------------------------------------------------------------------
struct Pkt {
    u8 *d;        // packet data (record header sits at d - 16)
    u32 caplen;   // current pcap caplen
    u32 len;      // current pcap len
    u32 phys;     // bytes from d that hold what the reference's buffer holds (its physical extent)
    u32 avail;    // bytes from d this lane may write (>= phys; slot tail or nothing)
    bool unsupported;
    u32 need;     // unsupported: the reference's buffer bytes [0, need) from d decide the output
    u32 ext;      // bytes from d the reference's buffer holds for this packet (its memcpy, the
                  // encoder's memmove, --fixlen=pad, fuzz writes): te_q8_replay's buffer view
    bool strict;  // te_q8_replay: a fuzz XOR of a byte past `phys` is a stale read too
    u32 room = 0;  // bytes before the record header (d - 16) that are this lane's: the slot's
                   // headroom, which an L2 push or a longer replacement header moves into.
                   // Tracked across every move of the record, so the two encodes of a fuzzed
                   // record (tcpedit.c:89,250-258) are bounded together, not each on its own
    u8 l2carry = 0;  // the en10mb encoder's dst_modified as the last C2S record left it (Q18)
    // Q18 under --fuzz-seed (the carry's mark run, LaunchArgs.q18_keys): this record's last
    // write of dst_modified -- bit 1 written, bit 0 the value -- and bit 2 once the record
    // went back to `again:` after the fuzz step (tcpedit.c:255)
    u8 q18ev = 0;
    // DLT_JUNIPER_ETHER: the decoder state the last whole inner decode before this record
    // left (jc), or none yet (jnone: zeros, the encoder's own extra) -- what a frame whose
    // extensions are not Ethernet is encoded with.  Neither: not at hand (fails loudly)
    const te_jstate_t *jc = nullptr;
    bool jnone = false;
    // ... and as this record's own first pass leaves it (its whole decode, else the same):
    // what the second decode of a fuzzed record reads when it is a warning frame
    const te_jstate_t *jc2 = nullptr;
    bool jnone2 = false;
    // the generic lane's tile (LDS) path: do_checksum leaves the L4 payload sum to the block
    // (all 256 threads sum every record's L4 bytes in 64-byte pieces) and records the job;
    // the lane writes the field once the block has summed (tile_body)
    bool defer = false;
    u8 *job_l4 = nullptr;   // first byte summed
    int job_len = 0;        // bytes summed (0: no job)
    u8 *job_field = nullptr;
    u32 job_base = 0;       // the pseudo header's sum, added to the payload's
};

// a read of bytes [.., end) from d that lie past the packet's physical bytes: the
// reference reads its static buffer there.  The record is
// flagged; te_q8_replay reproduces it over an emulated static buffer.
DI void stale(Pkt &pk, int end) {
    pk.unsupported = true;
    if (end > (int)pk.need) pk.need = (u32)end;
}
// a record the replay cannot reproduce either (slot headroom, not stale bytes)
constexpr u32 NEED_NEVER = 0xffffffffu;

// te_q8_replay (pk.strict): the packet start moved from old_d to pk.d (an L2 push, pop
// or replacement moves the head here, where the reference memmove's the rest).  Bring
// the buffer bytes past the packet's new extent along, so that pk.d + x is the
// reference's buffer offset x past the packet too: its memmove leaves them in place.
DI void strict_tail(Pkt &pk, const u8 *old_d) {
    if (!pk.strict) return;
    const u32 V = pk.phys;  // known bytes, in the old coordinates (phys not yet adjusted)
    if (pk.d < old_d)
        for (u32 x = pk.ext; x < V; ++x) pk.d[x] = old_d[x];
    else
        for (u32 x = V; x-- > pk.ext;) pk.d[x] = old_d[x];
    pk.phys = V > pk.ext ? V : pk.ext;
}

struct Dec {  // tcpeditdlt_t + en10mb_extra_t fields the encode/merge steps read
    u8 dstaddr[6], srcaddr[6];
    int proto;           // ctx->proto (network-order ethertype value)
    int proto_vlan_tag;  // ctx->proto_vlan_tag
    int l2offset, l2len;
    int vlan;
    u32 vlan_offset;
    u16 vlan_tag, vlan_pri, vlan_cfi, vlan_proto;
    bool dst_modified;   // en10mb_extra_t.dst_modified (read by the multicast MAC update)
    // DLT_JUNIPER_ETHER: the context's decoded extra is the en10mb sub-decoder's (a whole
    // inner decode copied it in, dlt_utils.c:262-263) -- too small for dlt_hdlc_encode
    bool jsub = false;
};

// ---------------------------------------------------------------------------
// L2 chain walk: get_l2len_protocol (src/common/get.c:262-451) for DLT_EN10MB,
// with parse_vlan (:170-182), parse_mpls (:87-157), parse_metadata (:196-236).
// Returns 0 and fills protocol/l2len/l2offset/vlan_offset, or -1.
// ---------------------------------------------------------------------------
struct L2 {
    u16 protocol;
    u32 l2len, l2offset, vlan_offset;
};

DI int get_l2len_protocol(const u8 *pkt, u32 datalen, L2 &r) {
    r.protocol = 0;
    r.l2len = 0;
    r.l2offset = 0;
    r.vlan_offset = 0;
    if (datalen == 0) return -1;
    u32 l2_net_off = 14;
    if (datalen <= l2_net_off + 4) return -1;
    u16 et = be16(pkt + 12);
    // bounded walk: every step consumes >= 4 bytes of a <= MAXPACKET buffer
    for (int guard = 0; guard < 65536; ++guard) {
        if (et == 0x8100 || et == 0x88A8 || et == 0x9100) {
            if (r.vlan_offset == 0) r.vlan_offset = l2_net_off;
            if (datalen < l2_net_off + 4) return -1;
            et = be16(pkt + l2_net_off + 2);
            l2_net_off += 4;
        } else if (et == 0x8847 || et == 0x8848) {
            u32 len = l2_net_off;
            bool bos = false;
            const u8 *lab = nullptr;
            while (!bos) {
                if ((uint64_t)len + 4 > datalen) return -1;
                lab = pkt + len;
                len += 4;
                u32 entry = be32(lab);
                bos = (entry & 0x100u) != 0;
                if ((entry >> 12) == 13) return -1;  // MPLS_LABEL_GACH
            }
            if ((u32)(lab + 4 - pkt) + 1 > datalen) return -1;
            u8 nib = lab[4] >> 4;
            if (nib == 4) {
                et = 0x0800;
            } else if (nib == 6) {
                et = 0x86DD;
            } else if (nib == 0) {  // EoMPLS: skip PW control word, inner Ethernet
                if ((uint64_t)len + 4 + 14 > datalen) return -1;
                len += 4;
                r.l2offset = len;
                et = be16(pkt + len + 12);
                len += 14;
            } else {
                return -1;
            }
            l2_net_off = len;
        } else {
            break;
        }
    }
    r.l2len = l2_net_off;
    if (et >= 1536) {
        r.protocol = et;
        return 0;
    }
    return -1;  // 802.3 length field / unsupported (get.c:367-380)
}

// get_l2len (get.c:456-470): 0 on failure
DI int get_l2len(const u8 *pkt, u32 datalen) {
    L2 r;
    if (get_l2len_protocol(pkt, datalen, r) == -1) return 0;
    return (int)r.l2len;
}

// dlt_en10mb_l2len (en10mb.c:917-943)
DI int en10mb_l2len(const u8 *pkt, int pktlen) {
    if (pktlen < 14) return -1;
    int l2 = get_l2len(pkt, (u32)pktlen);
    if (l2 > 0) return pktlen < l2 ? -1 : l2;
    return -1;
}

// ---------------------------------------------------------------------------
// L4 locators: get_layer4_v4 (get.c:611-625), get_ipv6_next (:757-800),
// get_layer4_v6 (:646-750), get_ipv6_l4proto (:806-853).  Offsets are byte
// offsets from the IP header; `end` is the offset of end_ptr.  -1 = NULL.
// ---------------------------------------------------------------------------
DI int l4_v4(const u8 *ip, int end) {
    int p = (ip[0] & 0x0f) << 2;
    return p > end ? -1 : p;
}

DI int ipv6_next(const u8 *ip, int ext, int end) {
    if (ext + 2 > end) return -1;
    switch (ip[ext]) {
        case 59: case 50: return -1;  // NO_NEXT, ESP
        case 44: return ext + 8 > end ? -1 : ext + 8;  // FRAGMENT: fixed 8 bytes
        case 41: case 43: case 60: case 0: case 51: {
            u8 extlen = (u8)(ip[ext + 1] * 4 + 8);  // IPV6_EXTLEN_TO_BYTES truncated to u8 (get.c:781)
            if (extlen == 0) return -1;
            return ext + extlen > end ? -1 : ext + extlen;
        }
        default: return ext;  // not an extension header: returns itself
    }
}

// get_layer4_v6.  Its NH_IPV6 case re-recurses with an unchanged proto until
// a call returns NULL (get.c:677-680 + :742-743), and every call advances the
// pointer by >= 40 bytes, so any v6-in-v6 header yields NULL.
DI int l4_v6(const u8 *ip, int base, int end) {
    int next = base + 40;
    if (next > end) return -1;
    u8 first = ip[base + 6];
    u8 proto = first;
    for (int guard = 0; guard < 4096; ++guard) {
        if (proto == 41) return -1;
        if (proto == 51 || proto == 43 || proto == 60 || proto == 0 || proto == 44) {
            int ex = ipv6_next(ip, next, end);
            if (ex < 0 || ex + 2 > end) return -1;
            proto = ip[ex];
            next = ex;
            continue;
        }
        if (proto == 50) return -1;  // ESP
        if (proto != first) {
            if (next + 2 > end) return -1;
            next = next + (ip[next + 1] * 4 + 8);  // not truncated here (get.c:728)
            if (next > end) return -1;
        }
        return next;
    }
    return -1;
}

DI u8 l4proto_v6(const u8 *ip, int end) {
    int base = 0;
    for (int depth = 0; depth < 64; ++depth) {
        int ptr = base + 40;
        if (ptr > end) return 59;
        u8 proto = ip[base + 6];
        bool recurse = false;
        for (int guard = 0; guard < 4096; ++guard) {
            if (proto == 59 || proto == 44 || proto == 50) return proto;
            if (proto == 41) {
                recurse = true;
                break;
            }
            if (proto == 51 || proto == 43 || proto == 60 || proto == 0) {
                int ex = ipv6_next(ip, ptr, end);
                if (ex < 0 || ex + 2 > end) return 59;
                proto = ip[ex];
                ptr = ex;
                continue;
            }
            return proto;
        }
        if (!recurse) return 59;
        base = ptr;
    }
    return 59;
}

// ---------------------------------------------------------------------------
// One's-complement sums (checksum.c:175-196 do_checksum_math semantics).
// The reference adds little-endian u16 loads relative to the start pointer
// (odd trailing byte as the low byte) into an int; only that sum's
// end-around-carry fold is observable, so we accumulate 32-bit words in a u64
// over aligned loads and fold, byte-swapping when the start is odd.
// ---------------------------------------------------------------------------
DI u32 fold16(unsigned long long s) {
    while (s >> 16) s = (s & 0xffffull) + (s >> 16);
    return (u32)s;
}

// sum of `len` bytes at p, weights relative to p (even offset -> low byte).
// Each dword adds as its two 16-bit words (v_sad_u16), which folds to the same
// one's-complement value as the dword sum (2^16 == 1 mod 0xffff, and both sums are 0 only
// for all-zero bytes).
DI u32 wsum_acc16(u32 x, u32 acc) {
#ifdef TE_HOST_EMU
    return acc + (x & 0xffffu) + (x >> 16);
#else
    return __builtin_amdgcn_sad_u16(x, 0u, acc);
#endif
}
// mask of bytes [lo, hi) of a dword, lo and hi clamped to [0, 4]
DI u32 dmask(int lo, int hi) {
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    const u32 mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
    const u32 ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
    return mh & ~ml;
}
#ifdef TE_HOST_EMU
DI u32 csum_bytes(const u8 *p, int len) {  // (host debugging harness: byte loop)
    if (len <= 0) return 0;
    const uintptr_t a = (uintptr_t)p;
    unsigned long long s = 0;
    for (int i = 0; i < len; ++i) s += (u32)p[i] << (8 * ((a + i) & 1));
    u32 f = fold16(s);
    if (a & 1) f = ((f >> 8) | (f << 8)) & 0xffff;
    return f;
}
#else
// The bytes are read as whole aligned 16-byte quads: the quad holding p, every quad up to
// the one holding p + len - 1, and no other.  Each load therefore lies inside the aligned
// 16-byte granule of a byte the packet owns -- it cannot cross a page, or reach past the
// end (or before the start) of the LDS tile or HBM scratch slot by more than that
// granule's other bytes -- and the first and last quads' bytes outside [p, p + len) are
// masked off.  (A 16-byte-load variant that read quads past the last one holding a packet
// byte is the one the round-2 notes record as faulting in the fast-lane tests; every load
// here is bounded by construction, and tests/test_gpu_parity.py puts huge records flush
// against the end of the image, the scratch slot and the output.)  One lane sums a whole
// packet, so the middle quads go four at a time, all in flight before the first add.
DI uint32_t quad_sum(const uint4 v, uint32_t acc) {
    return wsum_acc16(v.x, wsum_acc16(v.y, wsum_acc16(v.z, wsum_acc16(v.w, acc))));
}
DI uint32_t quad_sum_masked(const uint4 v, int off, int lo, int hi, uint32_t acc) {
    // bytes [lo, hi) of the quad run, quad byte 0 at run offset `off`
    return wsum_acc16(v.x & dmask(lo - off, hi - off),
                      wsum_acc16(v.y & dmask(lo - off - 4, hi - off - 4),
                                 wsum_acc16(v.z & dmask(lo - off - 8, hi - off - 8),
                                            wsum_acc16(v.w & dmask(lo - off - 12, hi - off - 12), acc))));
}
// the sum of bytes [p, p + len) with absolute weights (a byte at an even address is the
// low byte of its 16-bit word), unfolded: csum_bytes folds it and swaps for an odd p
DI unsigned long long sum_abs(const u8 *p, int len) {
    if (len <= 0) return 0;
    const int h = (int)((uintptr_t)p & 15u);  // p's byte within its quad
    const uint4 *Q = (const uint4 *)(p - h);   // (same granule as p: pointer arithmetic keeps the address space)
    const int hi = h + len;                    // run offsets [h, hi) are the packet's
    const int nq = (hi + 15) >> 4;             // quads 0 .. nq - 1
    unsigned long long s = quad_sum_masked(Q[0], 0, h, hi, 0u);
    int k = 1;
    for (; k + 4 <= nq - 1; k += 4) {  // 16 dwords x 0x1fffe: no u32 overflow
        const uint4 v0 = Q[k], v1 = Q[k + 1], v2 = Q[k + 2], v3 = Q[k + 3];
        s += quad_sum(v0, quad_sum(v1, quad_sum(v2, quad_sum(v3, 0u))));
    }
    for (; k < nq - 1; ++k) s += quad_sum(Q[k], 0u);
    if (nq > 1) s += quad_sum_masked(Q[nq - 1], 16 * (nq - 1), h, hi, 0u);
    return s;
}
DI u32 csum_bytes(const u8 *p, int len) {
    if (len <= 0) return 0;
    u32 f = fold16(sum_abs(p, len));
    if ((uintptr_t)p & 1u) f = ((f >> 8) | (f << 8)) & 0xffff;  // absolute -> relative weights
    return f;
}
#endif
// a deferred job's payload sum (the fold of its pieces' absolute-weight sums) -> the sum
// csum_bytes(job_l4, job_len) would have returned
DI u32 csum_of_job(const u8 *l4, u32 abs_sum) {
    u32 f = fold16(abs_sum);
    if ((uintptr_t)l4 & 1u) f = ((f >> 8) | (f << 8)) & 0xffff;
    return f;
}

// CHECKSUM_CARRY (checksum.h:25) applied to a plain non-negative sum
DI u16 csum_carry(unsigned long long x) { return (u16)(~fold16(x) & 0xffff); }

// ---------------------------------------------------------------------------
// RFC 1624 incremental updates: incremental_checksum.h:46-118, .c:40-118
// ---------------------------------------------------------------------------
DI u16 csum_fold32(u32 sum) {
    sum = (sum & 0xffff) + (sum >> 16);
    sum = (sum & 0xffff) + (sum >> 16);
    return (u16)~sum;
}
DI u32 csum_add(u32 c, u32 a) {
    u32 r = c + a;
    return r + (r < a);
}
DI u16 csum16_add(u16 c, u16 a) {
    u16 r = (u16)(c + a);
    return (u16)(r + (r < a));
}
// value forms (shared with the register-resident fast lane)
DI u16 csum_replace2_v(u16 s, u16 from, u16 to) { return (u16)~csum16_add(csum16_add((u16)~s, (u16)~from), to); }
DI u16 csum_replace4_v(u16 s, u32 from, u32 to) { return csum_fold32(csum_add(csum_add(~(u32)s, ~from), to)); }
DI u16 csum_replace16_v(u16 s, const u32 *from, const u32 *to) {
    // csum_partial over {~from[0..3], to[0..3]} (do_csum on an aligned 32-byte array)
    u32 result = 0, carry = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32 w = i < 4 ? ~from[i] : to[i - 4];
        result += carry;
        result += w;
        carry = (w > result);
    }
    result += carry;
    result = (result & 0xffff) + (result >> 16);
    result = (result & 0xffff) + (result >> 16);
    result = (result & 0xffff) + (result >> 16);
    u32 wsum = ~(u32)s;
    result += wsum;
    if (wsum > result) result += 1;
    return csum_fold32(result);
}
DI void csum_replace2(u8 *sp, u16 from, u16 to) { st16(sp, csum_replace2_v(ld16(sp), from, to)); }
DI void csum_replace4(u8 *sp, u32 from, u32 to) { st16(sp, csum_replace4_v(ld16(sp), from, to)); }
DI void csum_replace16(u8 *sp, const u8 *from, const u8 *to) {
    u32 f[4], t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[i] = ld32(from + 4 * i);
        t[i] = ld32(to + 4 * i);
    }
    st16(sp, csum_replace16_v(ld16(sp), f, t));
}

// ---------------------------------------------------------------------------
// Small predicates
// ---------------------------------------------------------------------------
// edit_packet.c:1204 (ntohl(ip) & 0xf0000000) == 0xe0000000, on the first octet = the low byte
DI bool mcast4(u32 ip_le) { return (ip_le & 0xf0u) == 0xe0u; }
DI bool mcast6(const u8 *a) { return a[0] == 0xff; }                                  // :1229

DI bool is_unicast_ethernet(const u8 *e) {  // plugins/ethernet.c:30-57
    if (e[0] == 0xff && e[1] == 0xff && e[2] == 0xff && e[3] == 0xff && e[4] == 0xff && e[5] == 0xff) return false;
    if (e[0] == 0x01 && e[1] == 0x00 && e[2] == 0x5e) return false;
    if (e[0] == 0x33 && e[1] == 0x33) return false;
    if (e[0] == 0x00 && e[1] == 0x00 && e[2] == 0x50 && e[3] == 0x00 && (e[4] == 0x01 || e[4] == 0x02))
        return false;  // IPV4_VRRP / IPV6_VRRP (defines.h.in:226-227)
    return true;
}

// ip_in_cidr (cidr.c:425-468): 64-bit mask semantics
DI bool ip_in_cidr(const te_cidr_t &c, u32 ip_le) {
    if (c.family != 4) return false;
    if (c.masklen == 0 && c.network == 0) return true;
    unsigned long long mask = ~0ull << (32 - c.masklen);
    return (((unsigned long long)bswap32(ip_le)) & mask) == (((unsigned long long)bswap32(c.network)) & mask);
}

// ip6_in_cidr (cidr.c:478-529)
DI bool ip6_in_cidr(const te_cidr_t &c, const u8 *a) {
    if (c.family != 6) return false;
    if (c.masklen == 0 && (ld32(a) | ld32(a + 4) | ld32(a + 8) | ld32(a + 12)) == 0) return true;
    u32 j = (u32)c.masklen / 8;
    for (u32 i = 0; i < j; ++i)
        if (a[i] != c.network6[i]) return false;
    u32 k = (u32)c.masklen % 8;
    if (k == 0) return true;
    k = ~0u << (8 - k);
    return (a[j] & k) == (c.network6[j] & k);
}

// remap_ipv4 (edit_packet.c:713-746); x86 masks a shift by 32 to 0
DI u32 remap_ipv4(const te_dev_cfg_t &cfg, const te_cidr_t &c, u32 orig) {
    if (c.family != 4) return 0;
    if (cfg.skip_broadcast && mcast4(orig)) return orig;
    u32 mask = 0xffffffffu << ((32 - c.masklen) & 31);
    u32 network = bswap32(c.network) & mask;
    mask ^= 0xffffffffu;
    return bswap32(network ^ (bswap32(orig) & mask));
}

// remap_ipv6 (edit_packet.c:748-779) incl. its out-of-range write for
// non-octet masks, with x86's 5-bit shift-count masking.
// Returns 0, or (the stray write would land past `room_after_addr`, the packet's
// physical bytes) 1 + the offset from addr it reads and writes.
DI int remap_ipv6(const te_dev_cfg_t &cfg, const te_cidr_t &c, u8 *addr, int room_after_addr) {
    if (c.family != 6) return 0;
    if (cfg.skip_broadcast && mcast6(addr)) return 0;
    u32 j = (u32)c.masklen / 8;
    for (u32 i = 0; i < j; ++i) addr[i] = c.network6[i];
    u32 k = (u32)c.masklen % 8;
    if (k == 0) return 0;
    k = ~0u << (8 - k);
    u32 i = addr[j] & k;
    if ((int)i >= room_after_addr) return 1 + (int)i;
    u32 s1 = (8u - k) & 31u, s2 = k & 31u;
    addr[i] = (u8)((c.network6[j] & (0xffu << s1)) | (addr[i] & (0xffu >> s2)));
    return 0;
}

// the tile path: leave the payload sum of [l4, l4 + n) to the block (Pkt.defer)
DI bool defer_sum(Pkt &pk, u8 *l4, int n, u8 *field, unsigned long long base) {
    if (!pk.defer) return false;
    pk.job_l4 = l4;
    pk.job_len = n;
    pk.job_field = field;
    pk.job_base = (u32)base;  // (pseudo header + length word: far below 2^32)
    return true;
}

// ---------------------------------------------------------------------------
// Full checksum: do_checksum (checksum.c:34-170).  `ip` = L3 header, `end` =
// offset of end_ptr.  Reads past the materialised slot mark the packet.
// ---------------------------------------------------------------------------
DI int do_checksum(Pkt &pk, u8 *ip, int proto, int len, int end) {
    if (len <= 0) return RC_ERROR;
    bool v6 = (ip[0] >> 4) == 6;
    int ip_hl;
    if (v6) {
        proto = l4proto_v6(ip, end);
        int l4 = l4_v6(ip, 0, end);
        if (l4 < 0) return RC_WARN;
        ip_hl = l4;
        len -= (ip_hl - 40);
    } else {
        ip_hl = (ip[0] & 0x0f) << 2;
    }
    // bytes this sum reads: [ip + ip_hl, ip + ip_hl + len); past `avail` only
    // zero padding may be read (fixlen pad); anything else is the reference's
    // stale static buffer (Q8) which a lane cannot see.
    const int ipoff = (int)(ip - pk.d);
    auto readable = [&](int nbytes) -> int {  // bytes past `phys` are the reference's stale buffer
        int lim = (int)pk.phys - (ipoff + ip_hl);
        if (nbytes > lim) stale(pk, ipoff + ip_hl + nbytes);
        return nbytes <= lim ? nbytes : (lim < 0 ? 0 : lim);
    };
    u8 *l4 = ip + ip_hl;
    unsigned long long sum = 0;
    switch (proto) {
        case 6:
        case 44: {  // IPPROTO_TCP, IPPROTO_TCP_V6FRAG (tcpr.h:655)
            if (len < 20) return RC_WARN;
            if (ipoff + ip_hl + 18 > (int)pk.phys) { stale(pk, ipoff + ip_hl + 18); return RC_OK; }
            st16(l4 + 16, 0);
            sum = v6 ? csum_bytes(ip + 8, 32) : csum_bytes(ip + 12, 8);
            sum += bswap16((u16)(6 + len));
            if (defer_sum(pk, l4, readable(len), l4 + 16, sum)) break;
            sum += csum_bytes(l4, readable(len));
            st16(l4 + 16, csum_carry(sum));
            break;
        }
        case 17: {
            if (len < 8) return RC_WARN;
            if (ipoff + ip_hl + 8 > (int)pk.phys) { stale(pk, ipoff + ip_hl + 8); return RC_OK; }
            if (ld16(l4 + 6) == 0) break;
            st16(l4 + 6, 0);
            sum = v6 ? csum_bytes(ip + 8, 32) : csum_bytes(ip + 12, 8);
            sum += bswap16((u16)(17 + len));
            if (defer_sum(pk, l4, readable(len), l4 + 6, sum)) break;
            sum += csum_bytes(l4, readable(len));
            st16(l4 + 6, csum_carry(sum));
            break;
        }
        case 1: {
            if (len < 4) return RC_WARN;
            if (ipoff + ip_hl + 4 > (int)pk.phys) { stale(pk, ipoff + ip_hl + 4); return RC_OK; }
            st16(l4 + 2, 0);
            if (v6) {
                // CHECKSUM_CARRY assigns its argument; the interim value lands in
                // icmp_sum and is summed with the payload (checksum.c:131-135)
                sum = csum_bytes(ip + 8, 32);
                u32 f = (u32)((sum >> 16) + (sum & 0xffff));
                sum = f;
                st16(l4 + 2, (u16)(~(f + (f >> 16)) & 0xffff));
            }
            if (defer_sum(pk, l4, readable(len), l4 + 2, sum)) break;
            sum += csum_bytes(l4, readable(len));
            st16(l4 + 2, csum_carry(sum));
            break;
        }
        case 58: {
            if (len < 8) return RC_WARN;
            if (ipoff + ip_hl + 4 > (int)pk.phys) { stale(pk, ipoff + ip_hl + 4); return RC_OK; }
            st16(l4 + 2, 0);
            if (v6) sum = csum_bytes(ip + 8, 32);
            sum += bswap16((u16)(58 + len));
            if (defer_sum(pk, l4, readable(len), l4 + 2, sum)) break;
            sum += csum_bytes(l4, readable(len));
            st16(l4 + 2, csum_carry(sum));
            break;
        }
        default:
            if (!v6) {
                st16(ip + 10, 0);
                st16(ip + 10, csum_carry(csum_bytes(ip, ip_hl)));
            } else {
                return RC_WARN;
            }
    }
    return RC_OK;
}

// fix_ipv4_checksums (edit_packet.c:55-112)
DI int fix_ipv4_checksums(Pkt &pk, u8 *ip, int l2len) {
    if (pk.caplen < 20u + (u32)l2len) return RC_WARN;
    if ((ip[0] >> 4) != 4) return RC_ERROR;
    int ret1 = 0, ret2;
    int ip_len = (int)be16(ip + 2);
    int end = (int)pk.caplen - l2len;
    if (pk.caplen == pk.len && (be16(ip + 6) & 0x3fff) == 0) {
        if (ip_len != (int)(pk.caplen - (u32)l2len)) return RC_WARN;
        ret1 = do_checksum(pk, ip, ip[9], ip_len - ((ip[0] & 0x0f) << 2), end);
        if (ret1 < 0) return RC_ERROR;
    }
    ret2 = do_checksum(pk, ip, 0, ip_len, end);
    if (ret2 < 0) return RC_ERROR;
    if (ret1 == RC_WARN || ret2 == RC_WARN) return RC_WARN;
    return RC_OK;
}

// ipv6_header_length (edit_packet.c:118-140)
DI int ipv6_header_length(Pkt &pk, const u8 *ip6, u32 pkt_len, int l2len) {
    int offset = 40;
    u8 nh = ip6[6];
    const int ipoff = (int)(ip6 - pk.d);
    for (int guard = 0; guard < 65536 && (u32)(2 + offset + l2len) < pkt_len; ++guard) {
        if (nh != 0 && nh != 43 && nh != 44) return offset;
        if (ipoff + offset + 2 > (int)pk.phys) { stale(pk, ipoff + offset + 2); return offset; }
        nh = ip6[offset];
        offset += (ip6[offset + 1] + 1) << 3;
    }
    return -1;
}

// fix_ipv6_checksums (edit_packet.c:142-189)
DI int fix_ipv6_checksums(Pkt &pk, u8 *ip6, int l2len) {
    if (pk.caplen < 40u + (u32)l2len) return RC_WARN;
    if ((ip6[0] >> 4) != 6) return RC_ERROR;
    int ret = 0;
    if (pk.caplen == pk.len) {
        int ip6_len = ipv6_header_length(pk, ip6, pk.len, l2len);
        if ((int)ld16(ip6 + 4) < ip6_len) return RC_WARN;  // raw network-order compare (:167)
        ret = do_checksum(pk, ip6, ip6[6], be16(ip6 + 4), (int)pk.caplen - l2len);
        if (ret < 0) return RC_ERROR;
    }
    return ret == RC_WARN ? RC_WARN : RC_OK;
}

// ipv4_addr_csum_replace (edit_packet.c:259-296)
DI void ipv4_addr_csum_replace(u8 *ip, u32 old_ip, u32 new_ip, int l3len) {
    int len = l3len;
    if (len < 20) return;
    csum_replace4(ip + 10, old_ip, new_ip);
    u8 proto = ip[9];
    int l4;
    if (proto == 17) {
        l4 = l4_v4(ip, l3len);
        len -= ((ip[0] & 0x0f) << 2) + 8;
    } else if (proto == 6) {
        l4 = l4_v4(ip, l3len);
        len -= ((ip[0] & 0x0f) << 2) + 20;
    } else {
        return;
    }
    if (l4 < 0 || len < 0) return;
    if ((be16(ip + 6) & 0x1fff) == 0) {
        if (proto == 6)
            csum_replace4(ip + l4 + 16, old_ip, new_ip);
        else if (ld16(ip + l4 + 6))
            csum_replace4(ip + l4 + 6, old_ip, new_ip);
    }
}

// ipv6_addr_csum_replace (edit_packet.c:298-330)
DI void ipv6_addr_csum_replace(Pkt &pk, u8 *ip6, const u8 *old_ip, const u8 *new_ip, int l3len) {
    if (l3len < 40) return;
    u8 proto = l4proto_v6(ip6, l3len);
    if (proto != 17 && proto != 6 && proto != 58) return;
    int l4 = l4_v6(ip6, 0, l3len);
    if (l4 < 0) return;
    int fld = proto == 6 ? 16 : (proto == 17 ? 6 : 2);
    if ((int)(ip6 - pk.d) + l4 + fld + 2 > (int)pk.phys) {  // past the physical packet: stale bytes
        stale(pk, (int)(ip6 - pk.d) + l4 + fld + 2);
        return;
    }
    if (proto == 17 && ld16(ip6 + l4 + 6) == 0) return;
    csum_replace16(ip6 + l4 + fld, old_ip, new_ip);
}

// randomize_ipv4_addr (edit_packet.c:336-357) without the skip test; s = bswap32(seed)
DI u32 randomize_ipv4_sw(u32 s, u32 ip) {
    const bool was = mcast4(ip);
    const u32 r = (ip ^ s) - (ip & s);
    // htonl((ntohl(r) & 0x0fffffff) | 0xe0000000) and htonl(ntohl(r) & 0x7fffffff),
    // on the first octet (the low byte of the little-endian value)
    const bool now = mcast4(r);
    const u32 r1 = (r & 0xffffff0fu) | 0xe0u, r2 = r & 0xffffff7fu;
    return (was && !now) ? r1 : ((!was && now) ? r2 : r);
}
DI u32 randomize_ipv4_addr(const te_dev_cfg_t &cfg, u32 ip) {
    if (cfg.skip_broadcast && mcast4(ip)) return ip;
    return randomize_ipv4_sw(bswap32(cfg.seed), ip);
}

// randomize_ipv6_addr (edit_packet.c:359-379)
DI void randomize_ipv6_addr(const te_dev_cfg_t &cfg, u8 *a) {
    bool was = mcast6(a);
    u32 s = bswap32(cfg.seed);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        u32 p = ld32(a + 4 * i);
        st32(a + 4 * i, (p ^ s) - (p & s));
    }
    if (was && !mcast6(a))
        a[0] = 0xff;
    else if (!was && mcast6(a))
        a[0] = 0xaa;
}

// rewrite_ports (portmap.c:267-330) with the first-match port map as a 64K LUT
DI int rewrite_ports(const u16 *lut, u8 proto, u8 *l4, int l4len) {
    int sumoff;
    if (proto == 6) {
        if (l4len < 20) return RC_WARN;
        sumoff = 16;
    } else if (proto == 17) {
        if (l4len < 8) return RC_WARN;
        sumoff = 6;
    } else {
        return 0;
    }
#pragma unroll
    for (int which = 0; which < 2; ++which) {  // destination port first, then source
        u8 *pp = l4 + (which == 0 ? 2 : 0);
        u16 oldp = ld16(pp);
        u16 np = lut[oldp];
        if (np != oldp) {
            if (proto == 6 || ld16(l4 + 6)) csum_replace2(l4 + sumoff, oldp, np);
            st16(pp, np);
        }
    }
    return 0;
}

// rewrite_seqs (rewrite_sequence.c:37-55)
DI void rewrite_seqs(Pkt &pk, const te_dev_cfg_t &cfg, u8 *tcp) {
    int off = (int)(tcp - pk.d);
    if (off + 18 > (int)pk.phys) {  // fields past the physical packet (stale bytes)
        stale(pk, off + 18);
        return;
    }
    u32 ns = be32(tcp + 4) + cfg.tcp_sequence_adjust;
    csum_replace4(tcp + 16, ld32(tcp + 4), bswap32(ns));
    st32(tcp + 4, bswap32(ns));
    if (!((tcp[13] & 0x02) && !(tcp[13] & 0x10))) {
        u32 na = be32(tcp + 8) + cfg.tcp_sequence_adjust;
        csum_replace4(tcp + 16, ld32(tcp + 8), bswap32(na));
        st32(tcp + 8, bswap32(na));
    }
}

// ---------------------------------------------------------------------------
// rewrite_ipv4l3 / rewrite_ipv6l3 (edit_packet.c:787-1019)
// ---------------------------------------------------------------------------
DI void rewrite_ipv4l3(const te_dev_cfg_t &cfg, u8 *ip, int dir, int len) {
    for (int m = 0; m < cfg.n_srcipmap; ++m) {
        const te_cidrmap_t &e = TE_CMAP(cfg, 2, m);
        if (ip_in_cidr(e.from, ld32(ip + 12))) {
            u32 o = ld32(ip + 12);
            st32(ip + 12, remap_ipv4(cfg, e.to, o));
            ipv4_addr_csum_replace(ip, o, ld32(ip + 12), len);
            break;
        }
    }
    for (int m = 0; m < cfg.n_dstipmap; ++m) {
        const te_cidrmap_t &e = TE_CMAP(cfg, 3, m);
        if (ip_in_cidr(e.from, ld32(ip + 16))) {
            u32 o = ld32(ip + 16);
            st32(ip + 16, remap_ipv4(cfg, e.to, o));
            ipv4_addr_csum_replace(ip, o, ld32(ip + 16), len);
            break;
        }
    }
    if (cfg.n_cidrmap1 == 0) return;
    const int w1 = dir == TE_DIR_C2S ? 0 : 1, w2 = 1 - w1;
    int n1 = dir == TE_DIR_C2S ? cfg.n_cidrmap1 : cfg.n_cidrmap2;
    int n2 = dir == TE_DIR_C2S ? cfg.n_cidrmap2 : cfg.n_cidrmap1;
    int i1 = 0, i2 = 0;
    bool didsrc = false, diddst = false;
    for (;;) {
        const te_cidrmap_t &e2 = TE_CMAP(cfg, w2, i2), &e1 = TE_CMAP(cfg, w1, i1);
        if (!diddst && ip_in_cidr(e2.from, ld32(ip + 16))) {
            u32 o = ld32(ip + 16);
            st32(ip + 16, remap_ipv4(cfg, e2.to, o));
            ipv4_addr_csum_replace(ip, o, ld32(ip + 16), len);
            diddst = true;
        }
        if (!didsrc && ip_in_cidr(e1.from, ld32(ip + 12))) {
            u32 o = ld32(ip + 12);
            st32(ip + 12, remap_ipv4(cfg, e1.to, o));
            ipv4_addr_csum_replace(ip, o, ld32(ip + 12), len);
            didsrc = true;
        }
        if (!(diddst && didsrc) && !(i1 + 1 >= n1 && i2 + 1 >= n2)) {
            if (i1 + 1 < n1) ++i1;
            if (i2 + 1 < n2) ++i2;
        } else {
            break;
        }
    }
}

DI void rewrite_ipv6_addr_pair(Pkt &pk, const te_dev_cfg_t &cfg, const te_cidr_t &to, u8 *ip6, int aoff, int l3len) {
    u8 old[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) old[b] = ip6[aoff + b];
    int room = (int)pk.phys - ((int)(ip6 - pk.d) + aoff);
    const int r = remap_ipv6(cfg, to, ip6 + aoff, room);
    if (r) stale(pk, (int)(ip6 - pk.d) + aoff + r);
    ipv6_addr_csum_replace(pk, ip6, old, ip6 + aoff, l3len);
}

DI void rewrite_ipv6l3(Pkt &pk, const te_dev_cfg_t &cfg, u8 *ip6, int dir, int l3len) {
    // the ICMPv6-error recursion (:988-1013) is walked iteratively
    for (int depth = 0; depth < 64; ++depth) {
        for (int m = 0; m < cfg.n_srcipmap; ++m) {
            const te_cidrmap_t &e = TE_CMAP(cfg, 2, m);
            if (ip6_in_cidr(e.from, ip6 + 8)) {
                rewrite_ipv6_addr_pair(pk, cfg, e.to, ip6, 8, l3len);
                break;
            }
        }
        for (int m = 0; m < cfg.n_dstipmap; ++m) {
            const te_cidrmap_t &e = TE_CMAP(cfg, 3, m);
            if (ip6_in_cidr(e.from, ip6 + 24)) {
                rewrite_ipv6_addr_pair(pk, cfg, e.to, ip6, 24, l3len);
                break;
            }
        }
        if (cfg.n_cidrmap1 != 0) {
            const int w1 = dir == TE_DIR_C2S ? 0 : 1, w2 = 1 - w1;
            int n1 = dir == TE_DIR_C2S ? cfg.n_cidrmap1 : cfg.n_cidrmap2;
            int n2 = dir == TE_DIR_C2S ? cfg.n_cidrmap2 : cfg.n_cidrmap1;
            int i1 = 0, i2 = 0;
            bool didsrc = false, diddst = false;
            for (;;) {
                const te_cidrmap_t &e2 = TE_CMAP(cfg, w2, i2), &e1 = TE_CMAP(cfg, w1, i1);
                if (!diddst && ip6_in_cidr(e2.from, ip6 + 24)) {
                    rewrite_ipv6_addr_pair(pk, cfg, e2.to, ip6, 24, l3len);
                    diddst = true;
                }
                if (!didsrc && ip6_in_cidr(e1.from, ip6 + 8)) {
                    rewrite_ipv6_addr_pair(pk, cfg, e1.to, ip6, 8, l3len);
                    didsrc = true;
                }
                if (!(diddst && didsrc) && !(i1 + 1 >= n1 && i2 + 1 >= n2)) {
                    if (i1 + 1 < n1) ++i1;
                    if (i2 + 1 < n2) ++i2;
                } else {
                    break;
                }
            }
        }
        if (l3len <= 0) return;
        if (l4proto_v6(ip6, l3len) != 58) return;
        int ic = l4_v6(ip6, 0, l3len);
        if (ic < 0 || ic + 8 > l3len) return;
        u8 type = ip6[ic];
        if (type < 1 || type > 4) return;  // ICMP6_UNREACH..ICMP6_PARAMPROB
        u8 *emb = ip6 + ic + 8;
        int emb_len = l3len - (ic + 8);
        if (!(emb_len >= 40 && (emb[0] >> 4) == 6)) return;
        ip6 = emb;
        l3len = emb_len;
    }
}

// randomize_iparp (edit_packet.c:1025-1083) / rewrite_iparp (:1093-1198)
DI bool arp_addrs(Pkt &pk, u8 *arp, u8 **ip1, u8 **ip2) {
    int base = (int)(arp - pk.d);
    if (base + 8 > (int)pk.phys) {  // ARP header past the physical packet
        stale(pk, base + 8);
        return false;
    }
    if (be16(arp + 2) != 0x0800) return false;
    u16 op = be16(arp + 6);
    if (op != 1 && op != 2) return false;
    int o1 = 8 + arp[4];
    int o2 = o1 + arp[5] + arp[4];
    if (base + o2 + 4 > (int)pk.phys) {  // address bytes past the physical packet
        stale(pk, base + o2 + 4);
        return false;
    }
    *ip1 = arp + o1;
    *ip2 = arp + o2;
    return true;
}

DI void rewrite_iparp(Pkt &pk, const te_dev_cfg_t &cfg, u8 *arp, int dir) {
    int w1 = 0, w2 = 1, n1 = 0, n2 = 0;
    if (dir == TE_DIR_C2S) {
        n1 = cfg.n_cidrmap1; n2 = cfg.n_cidrmap2;
    } else if (dir == TE_DIR_S2C) {
        w1 = 1; w2 = 0; n1 = cfg.n_cidrmap2; n2 = cfg.n_cidrmap1;
    }
    if (n1 == 0 || n2 == 0) return;
    u8 *ip1, *ip2;
    if (!arp_addrs(pk, arp, &ip1, &ip2)) return;
    bool request = be16(arp + 6) == 1;
    int i1 = 0, i2 = 0;
    bool didsrc = false, diddst = false;
    for (;;) {
        u8 *dsta = request ? ip1 : ip2, *srca = request ? ip2 : ip1;
        const te_cidrmap_t &e2 = TE_CMAP(cfg, w2, i2), &e1 = TE_CMAP(cfg, w1, i1);
        if (!diddst && ip_in_cidr(e2.from, ld32(dsta))) {
            st32(dsta, remap_ipv4(cfg, e2.to, ld32(dsta)));
            diddst = true;
        }
        if (!didsrc && ip_in_cidr(e1.from, ld32(srca))) {
            st32(srca, remap_ipv4(cfg, e1.to, ld32(srca)));
            didsrc = true;
        }
        if (!(diddst && didsrc) && !(i1 + 1 >= n1 && i2 + 1 >= n2)) {
            if (i1 + 1 < n1) ++i1;
            if (i2 + 1 < n2) ++i2;
        } else {
            break;
        }
    }
}

// untrunc_packet (edit_packet.c:526-621).  Returns -1 (error), 0, 1.
DI int untrunc_packet(Pkt &pk, const te_dev_cfg_t &cfg, u8 *ip, u8 *ip6) {
    if (pk.caplen == pk.len || (ip == nullptr && ip6 == nullptr))
        if (!cfg.mtu_truncate) return 0;
    int l2len = en10mb_l2len(pk.d, (int)pk.caplen);  // layer2len() via the encoder (dlt.c:165-172)
    if (l2len < 0) return -1;
    int chksum = 1;
    if (ip) {
        u16 off = be16(ip + 6);
        if (off & 0x1fff) {
            chksum = 0;
        } else if (ip[9] == 17 && (off & 0x2000)) {
            int f = (int)(ip - pk.d) + ((ip[0] & 0x0f) << 2) + 6;
            if (f + 2 > (int)pk.phys) stale(pk, f + 2);
            else st16(pk.d + f, 0);
            chksum = 0;
        }
    }
    if (cfg.fixlen == TE_FIXLEN_PAD) {
        if (pk.len > pk.caplen) {
            // memset(packet + caplen, 0, len - caplen): the tile sized this slot
            // for max(caplen, len) when --fixlen=pad is set
            if (pk.len > pk.avail) stale(pk, (int)NEED_NEVER);
            for (u32 i = pk.caplen; i < pk.avail && i < pk.len; ++i) pk.d[i] = 0;
            if (pk.len > pk.phys) pk.phys = pk.len < pk.avail ? pk.len : pk.avail;
            if (pk.len > pk.ext) pk.ext = pk.len;
            pk.caplen = pk.len;
        } else if (pk.len < pk.caplen) {
            return -1;
        }
    } else if (cfg.fixlen == TE_FIXLEN_TRUNC) {
        if (ip && pk.len != pk.caplen) st16(ip + 2, bswap16((u16)(pk.caplen - (u32)l2len)));
        pk.len = pk.caplen;
    } else if (cfg.mtu_truncate) {
        if (pk.len > (u32)(cfg.mtu + l2len)) {
            pk.len = pk.caplen = (u32)l2len + (u32)cfg.mtu;
            if (ip) st16(ip + 2, bswap16((u16)cfg.mtu));
            else if (ip6) st16(ip6 + 4, bswap16((u16)(cfg.mtu - 40)));
            else chksum = 0;
        }
    } else {
        return -1;  // "Invalid fixlen value" (TCPEDIT_FIXLEN_DEL lands here)
    }
    return chksum;
}

// ---------------------------------------------------------------------------
// DLT_EN10MB decode/encode/merge (plugins/dlt_en10mb/en10mb.c:402-887)
// ---------------------------------------------------------------------------
DI int en10mb_decode(const u8 *pkt, int pktlen, Dec &s) {
    L2 r;
    if (get_l2len_protocol(pkt, (u32)pktlen, r) == -1) return RC_ERROR;
    if ((u32)pktlen < 14 + r.l2offset) return RC_ERROR;
    const u8 *eth = pkt + r.l2offset;
    u16 prot = be16(eth + 12);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        s.dstaddr[i] = eth[i];
        s.srcaddr[i] = eth[6 + i];
    }
    s.proto_vlan_tag = prot;
    if (r.vlan_offset != 0) {
        if (r.vlan_offset != r.l2offset + 14) return RC_ERROR;  // VLAN after MPLS
        if ((u32)pktlen < r.vlan_offset + 4) return RC_ERROR;
        u16 tci = be16(pkt + r.vlan_offset);
        s.vlan = 1;
        s.vlan_offset = r.vlan_offset;
        s.vlan_proto = be16(pkt + r.vlan_offset + 2);
        s.vlan_tag = tci & 0x0fff;
        s.vlan_pri = tci & 0xe000;
        s.vlan_cfi = tci & 0x1000;
    } else {
        s.vlan = 0;
        s.vlan_offset = r.l2offset + 14;
        s.vlan_proto = prot;
    }
    s.proto = bswap16(prot);
    s.l2offset = (int)r.l2offset;
    s.l2len = (int)r.l2len;
#if defined(__HIP_DEVICE_COMPILE__)
    // Optimisation barrier.  Without it the gfx950 backend (ROCm 7.2, -O1..-O3)
    // re-materialises l2offset as 0 in en10mb_encode for EoMPLS frames whose
    // inner Ethernet carries an 802.1Q tag (test.pcap records 142/150/157/170/
    // 174-179), writing the inner MACs over the outer ones; the host build of
    // this same code is correct.  Pinning the decoded offsets in VGPRs costs nothing.
    asm volatile("" : "+v"(s.l2offset), "+v"(s.vlan_offset), "+v"(s.l2len));
#endif
    return RC_OK;
}

// ---------------------------------------------------------------------------
// The other decoders (src/tcpedit/plugins/dlt_*): plugin_proto and plugin_decode.
// ---------------------------------------------------------------------------
constexpr int RC_PROTO_SOFT = -2;  // TCPEDIT_SOFT_ERROR from a proto function (pppserial)

// dlt_null_proto (null.c:206-236, DLT_NULL and DLT_LOOP): the address family in either
// byte order (PF_INET6 is 10 here; the BSDs' 24/28/30 are taken too)
DI int null_proto(const u8 *p, u32 caplen) {
    if (caplen < 4) return RC_ERROR;
    const u32 af = ld32(p), saf = bswap32(af);
    if (af == 2 || saf == 2) return 0x0008;  // htons(ETHERTYPE_IP)
    if (af == 10 || saf == 10 || af == 24 || saf == 24 || af == 28 || saf == 28 || af == 30 || saf == 30)
        return 0xDD86;  // htons(ETHERTYPE_IP6)
    return RC_ERROR;
}
// dlt_raw_proto (raw.c:206-231): the IP version nibble
DI int raw_proto(const u8 *p, u32 caplen) {
    if (caplen < 20) return RC_ERROR;
    return (p[0] >> 4) == 4 ? 0x0008 : (p[0] >> 4) == 6 ? 0xDD86 : RC_ERROR;
}
// a byte the reference reads at packet offset `off` whatever the captured length: past the
// record's physical bytes it reads its static buffer (Q8: flagged, replayed)
DI u32 byte_at(Pkt &pk, int off) {
    if (off + 1 > (int)pk.phys) stale(pk, off + 1);
    return off < (int)pk.avail ? pk.d[off] : 0u;
}
// dlt_en10mb_proto (en10mb.c:741-762) of the Ethernet frame at p
DI int en10mb_proto_at(const u8 *p, u32 n) {
    if (n < 14) return RC_ERROR;
    L2 r;
    if (get_l2len_protocol(p, n, r) == -1) return RC_ERROR;
    return bswap16(r.protocol);
}

// DLT_IEEE802_11 (plugins/dlt_ieee80211): the frame control word is read with ntohs, so
// the masks of ieee80211_types.h:33-76 apply to (byte0 << 8 | byte1)
DI u32 w80211_fc(const u8 *d) { return (u32)d[0] << 8 | d[1]; }
DI int w80211_hdr(u32 fc, bool qos) { return (qos ? 2 : 0) + ((fc & 3u) == 3u ? 30 : 24); }  // + QoS, 4 addresses
// dlt_ieee80211_l2len (ieee80211.c:333-371): 0, not -1, for a short frame
DI int w80211_l2len(const u8 *d, int n) {
    if (n < 2) return 0;
    const u32 fc = w80211_fc(d);
    int h = w80211_hdr(fc, (fc & 0x8000u) == 0x8000u);
    if (n >= h + 8) h += d[h] == 0xAA && d[h + 1] == 0xAA ? 8 : 3;  // 802.2 SNAP or 802.2
    return n < h ? 0 : h;
}
// dlt_ieee80211_proto (ieee80211.c:246-291): the SNAP type, read at its offset whatever the
// captured length
DI int w80211_proto(Pkt &pk) {
    const u32 fc = byte_at(pk, 0) << 8 | byte_at(pk, 1);
    if ((fc & 0x0F00u) != 0x0800u) return RC_PROTO_SOFT;  // not a data frame
    const int h = w80211_hdr(fc, (fc & 0x8000u) == 0x8000u);
    if (byte_at(pk, h) == 0xAA && byte_at(pk, h + 1) == 0xAA) return (int)(byte_at(pk, h + 6) | byte_at(pk, h + 7) << 8);
    return RC_PROTO_SOFT;
}

// dlt_jnpr_ether_decode's header checks (jnpr_ether.c:215-273): RC_ERROR, JNPR_WARN (the
// extensions do not say Ethernet: media type 1 and encapsulation 14) or RC_OK; hl = the
// Juniper header's length (set for a warning too)
constexpr int JNPR_WARN = 1;
DI int jnpr_header(const u8 *d, u32 n, u32 &hl) {
    if (n < 6) return RC_ERROR;
    if (d[0] != 0x4d || d[1] != 0x47 || d[2] != 0x43) return RC_ERROR;  // JUNIPER_ETHER_MAGIC
    if (!(d[3] & 0x80)) return RC_ERROR;                                 // no L2 header
    hl = ((u32)d[4] << 8 | d[5]) + 6u;
    if (n < hl + 14) return RC_ERROR;
    // the extension TLVs: media type (3) and encapsulation (6), first byte of each value
    u32 ext = 6, dlt = 0, enc = 0;
    while (ext + 2 < hl) {
        const u32 el = d[ext + 1];
        if (d[ext] == 3) dlt = d[ext + 2];
        else if (d[ext] == 6) enc = d[ext + 2];
        if (dlt && enc) break;
        ext += el + 2;
    }
    if (ext > hl) return RC_ERROR;
    return dlt != 1 || enc != 14 ? JNPR_WARN : RC_OK;
}

// the decoder's proto (tcpedit_dlt_proto on the source DLT, tcpedit.c:96): the ethertype
// as the little-endian u16 of its network-order bytes, or < 0
DI int decoder_proto(Pkt &pk, const te_dev_cfg_t &cfg) {
    const u8 *d = pk.d;
    const u32 n = pk.caplen;
    switch (cfg.decoder) {
    case TE_DEC_JNPR: {  // dlt_jnpr_ether_proto (jnpr_ether.c:310-345): the inner frame's
        if (n < 6 || !(d[3] & 0x80)) return RC_ERROR;  // JUNIPER_ETHER_L2PRESENT
        const u32 hl = ((u32)d[4] << 8 | d[5]) + 6u;
        if (hl > n) return RC_ERROR;
        return en10mb_proto_at(d + hl, n - hl);
    }
    case TE_DEC_80211: return w80211_proto(pk);
    // radiotap.c:134-155, 344-364: the 802.11 frame is copied into the plugin's MAXPACKET
    // extra buffer only when at least that long, which no record is -- the 802.11 proto
    // reads zeros there, not a data frame: every record is a soft error
    case TE_DEC_RADIOTAP: return RC_PROTO_SOFT;
    case TE_DEC_SLL: return n < 16 ? RC_ERROR : (int)ld16(d + 14);  // linuxsll.c:213-226
    case TE_DEC_SLL2: return n < 20 ? RC_ERROR : (int)ld16(d);      // linuxsll2.c:226-238
    case TE_DEC_RAW: return raw_proto(d, n);
    case TE_DEC_NULL: return null_proto(d, n);
    // pppserial.c:257-281: the ethertype in host order (0x0800), which tcpedit.c:123,149
    // never take for IPv4; anything but PPP's IPv4 protocol is a soft error
    case TE_DEC_PPP: return n < 4 ? RC_ERROR : be16(d + 2) == 0x0021 ? 0x0800 : RC_PROTO_SOFT;
    case TE_DEC_CHDLC: return n < 4 ? RC_ERROR : (int)ld16(d + 2);  // hdlc.c:299-311
    default: return en10mb_proto_at(d, n);  // dlt_en10mb_proto
    }
}
// the decoder (plugin_decode) for the non-Ethernet DLTs: l2len, proto and, for the Linux
// cooked headers, the source address.  None of them sets the en10mb extra fields, which
// keep the zeroed start of the decoder's (larger) extra buffer (en10mb.c:100-110) --
// except the Juniper decoder, whose en10mb sub-decoder's extra becomes the encoder's.
// (A soft error from the decoder is returned as RC_ERROR: both make the record RC_SOFT.)
DI int foreign_decode(Pkt &pk, const te_dev_cfg_t &cfg, Dec &s) {
    const u8 *d = pk.d;
    const u32 n = pk.caplen;
#pragma unroll
    for (int i = 0; i < 6; ++i) s.dstaddr[i] = s.srcaddr[i] = 0;
    s.proto_vlan_tag = 0;
    s.l2offset = 0;
    s.vlan = 0;
    s.vlan_offset = 0;
    s.vlan_tag = s.vlan_pri = s.vlan_cfi = s.vlan_proto = 0;
    switch (cfg.decoder) {
    case TE_DEC_SLL:     // linuxsll.c:170-194
    case TE_DEC_SLL2: {  // linuxsll2.c:181-205
        const bool sll = cfg.decoder == TE_DEC_SLL;
        const u32 hl = sll ? 16u : 20u;
        if (n < hl) return RC_ERROR;
        s.proto = ld16(d + (sll ? 14 : 0));
        s.l2len = (int)hl;
        const u16 type = be16(d + (sll ? 2 : 8));
        if (type != 1 && type != 772) return RC_ERROR;  // ARPHRD_ETHER, ARPHRD_LOOPBACK
#pragma unroll
        for (int i = 0; i < 6; ++i) s.srcaddr[i] = d[(sll ? 6 : 12) + i];
        return RC_OK;
    }
    case TE_DEC_RAW: {  // raw.c:170-190
        if (n == 0) return RC_ERROR;
        const int p = raw_proto(d, n);
        if (p < 0) return RC_ERROR;
        s.proto = p;
        s.l2len = 0;
        return RC_OK;
    }
    case TE_DEC_NULL: {  // null.c:171-187
        const int p = null_proto(d, n);
        if (p < 0) return RC_ERROR;
        s.proto = p;
        s.l2len = 4;
        return RC_OK;
    }
    case TE_DEC_PPP:  // pppserial.c:196-231
        if (n < 4) return RC_ERROR;
        s.proto = be16(d + 2) == 0x0021 ? 0x0008 : (int)ld16(d + 2);
        s.l2len = 4;
        return RC_OK;
    case TE_DEC_JNPR: {  // dlt_jnpr_ether_decode (jnpr_ether.c:201-282)
        u32 hl = 0;
        const int h = jnpr_header(d, n, hl);
        if (h == RC_ERROR) return RC_ERROR;
        if (h == JNPR_WARN) {
            // TCPEDIT_WARN (:269-272): the header length is set, and the frame is encoded
            // with the state the last whole inner decode left in the context (the copied
            // addresses and proto, the sub-decoder's extra by pointer)
            if (pk.jc) {
                const te_jstate_t &c = *pk.jc;
                s.jsub = true;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    s.dstaddr[i] = c.dstaddr[i];
                    s.srcaddr[i] = c.srcaddr[i];
                }
                s.proto = c.proto;
                s.vlan = c.vlan;
                s.vlan_offset = c.vlan_offset;
                s.vlan_tag = c.vlan_tag;
                s.vlan_pri = c.vlan_pri;
                s.vlan_cfi = c.vlan_cfi;
                s.vlan_proto = c.vlan_proto;
            } else if (pk.jnone) {  // no whole decode yet: the zeroed context and extra
                s.proto = 0;
            } else {  // the carried state is not at hand: the record fails the run loudly
                stale(pk, (int)NEED_NEVER);
                return RC_ERROR;
            }
            s.l2len = (int)hl;
            return RC_OK;
        }
        // the en10mb sub-decoder works on a context of its own (jnpr_ether.c:135-136,276):
        // a decode that fails part-way leaves ours as it was; a whole one is copied in
        // (tcpedit_dlt_copy_decoder_state, dlt_utils.c:249-271: its addresses, proto and
        // extra; the l2lens add; ctx->l2offset stays 0)
        Dec t = s;
        if (en10mb_decode(d + hl, (int)(n - hl), t) == RC_ERROR) return RC_ERROR;
        t.l2len += (int)hl;
        t.l2offset = 0;
        // the first whole decode makes the sub-decoder's extra the encoder's: a fresh
        // dst_modified (en10mb_decode never writes it)
        if (pk.jnone) {
            t.dst_modified = false;
            pk.q18ev = (u8)((pk.q18ev & 4u) | 2u);
        }
        t.jsub = true;
        t.proto_vlan_tag = s.proto_vlan_tag;  // (the sub-context's: not copied, dlt_utils.c:254-263)
        s = t;
        return RC_OK;
    }
    case TE_DEC_80211: {  // dlt_ieee80211_decode (ieee80211.c:184-224)
        const int l2 = w80211_l2len(d, (int)n);
        const u32 fc = n >= 2 ? w80211_fc(d) : 0u;  // (n < 2: the proto was a stale read already)
        bool data;                                    // ieee80211_is_data (ieee80211_hdr.c:36-92)
        if (n <= 24) {
            data = false;
        } else if ((fc & 0xF000u) == 0xC000u || (fc & 0x0F00u) == 0x0800u) {
            data = true;
        } else {
            const int h = w80211_hdr(fc, (fc & 0xF000u) >= 0x8000u);
            data = (int)n >= h + 8 && d[h] == 0xAA && d[h + 1] == 0xAA;
        }
        if (!data) return RC_ERROR;                       // TCPEDIT_SOFT_ERROR
        if (n >= 24 && (fc & 0x40u)) return RC_ERROR;     // encrypted: TCPEDIT_SOFT_ERROR
        s.l2len = l2;
        // ieee80211_get_src/dst (ieee80211_hdr.c:120-184): by the DS bits
        const int ds = (int)(fc & 3u);
        const int so = ds == 3 ? 24 : ds == 2 ? 16 : 10, dof = ds == 3 ? 16 : ds == 2 ? 4 : 16;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            s.srcaddr[i] = (u8)byte_at(pk, so + i);
            s.dstaddr[i] = (u8)byte_at(pk, dof + i);
        }
        s.proto = w80211_proto(pk);
        return RC_OK;
    }
    case TE_DEC_RADIOTAP: return RC_ERROR;  // (its proto stops every record first)
    default:  // TE_DEC_CHDLC, hdlc.c:192-218 (its address/control extras are never marked filled)
        if (n < 4) return RC_ERROR;
        s.proto = ld16(d + 2);
        s.l2len = 4;
        return RC_OK;
    }
}

// subsmac and the MAC seed over the new Ethernet addresses (en10mb.c:662-690)
DI void en10mb_mac_rules(const te_dev_cfg_t &cfg, u8 *dh, u8 *sh) {
    for (int e = 0; e < cfg.n_subs; ++e) {
        const u8 *t = cfg.subs[e], *rw = cfg.subs[e] + 6;
        bool md = true, ms = true;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            md &= dh[i] == t[i];
            ms &= sh[i] == t[i];
        }
        if (md)
            for (int i = 0; i < 6; ++i) dh[i] = rw[i];
        if (ms)
            for (int i = 0; i < 6; ++i) sh[i] = rw[i];
    }
    if (cfg.random_set) {
        int us = is_unicast_ethernet(sh), ud = is_unicast_ethernet(dh);
        for (int i = cfg.random_keep; i < 6; ++i) {
            int ms = cfg.random_mask[i] * us, md = cfg.random_mask[i] * ud;
            sh[i] = (u8)((sh[i] ^ ms) - (sh[i] & ms));  // MAC_MASK_APPLY (en10mb.h:29-30)
            dh[i] = (u8)((dh[i] ^ md) - (dh[i] & md));
        }
        if (!cfg.random_keep) {
            sh[0] &= (u8)~(0x01 * us);
            dh[0] &= (u8)~(0x01 * ud);
        }
    }
}

DI bool l2_replace(Pkt &pk, int l2len, int n);
DI void l2_half_move(Pkt &pk, int oldl2, int newl2, int pktlen);

// dlt_en10mb_encode for another decoder (en10mb.c:544-548 and on): a 14-byte Ethernet
// header replaces the decoded one (the host refuses VLAN add here, and the configs where
// an address is missing, which the reference fails after its memmove).  Addresses:
// the options', else -- the Linux cooked headers' ETHERNET address type -- the decoded
// source and the context's never-set (zero) destination.  A C2S record without
// --enet-dmac sets dst_modified (its old first 6 bytes against that zero destination).
DI int en10mb_encode_foreign(Pkt &pk, const te_dev_cfg_t &cfg, Dec &s, int pktlen, int dir) {
    if (pktlen < 14) return RC_ERROR;
    // :518-521 (before anything moves): a tag to push, or the decoder's tagged frame
    if (cfg.vlan == TE_VLAN_ADD && !s.vlan && cfg.vlan_tag == 65535) return RC_ERROR;
    const int newl2 = cfg.vlan == TE_VLAN_ADD ? 18 : 14;  // :545-549
    if (pktlen < newl2 || pktlen + newl2 - s.l2len > MAXPACKET) return RC_ERROR;
    if (pktlen < s.l2len) return RC_ERROR;
    if (dir != TE_DIR_C2S && dir != TE_DIR_S2C) return RC_ERROR;
    const bool eth_addr = TE_DEC_ETH_ADDR(cfg.decoder);
    const bool c2s = dir == TE_DIR_C2S;
    const int sm = c2s ? TE_MASK_SMAC1 : TE_MASK_SMAC2, dm = c2s ? TE_MASK_DMAC1 : TE_MASK_DMAC2;
    const u8 *smac = c2s ? cfg.intf1_smac : cfg.intf2_smac;
    const u8 *dmac = c2s ? cfg.intf1_dmac : cfg.intf2_dmac;
    if (!eth_addr && (!(cfg.mac_mask & sm) || !(cfg.mac_mask & dm))) {
        // no address to fall back on (:599-602, :616-619): an error after the memmove, the
        // source address written first when only the destination is missing
        l2_half_move(pk, s.l2len, newl2, pktlen);
        if (cfg.mac_mask & sm)
#pragma unroll
            for (int i = 0; i < 6; ++i) pk.d[6 + i] = smac[i];
        return RC_ERROR;
    }
    bool old_nz = false;  // memcmp(eth->ether_dhost, ctx->dstaddr, 6) before the writes
#pragma unroll
    for (int i = 0; i < 6; ++i) old_nz |= pk.d[i] != s.dstaddr[i];
    // a VLAN push's bytes [14, 18) are the packet's before the memmove (:577 writes from
    // byte 18 on; pktlen >= 18 here) unless the tag lands there
    u8 pre[4];
    if (cfg.vlan == TE_VLAN_ADD)
#pragma unroll
        for (int i = 0; i < 4; ++i) pre[i] = pk.d[14 + i];
    if (!l2_replace(pk, s.l2len, newl2)) return RC_ERROR;
    if (cfg.vlan == TE_VLAN_ADD)
#pragma unroll
        for (int i = 0; i < 4; ++i) pk.d[14 + i] = pre[i];
    pktlen += newl2 - s.l2len;
    u8 *dh = pk.d, *sh = pk.d + 6;
    const bool l2skip = cfg.l2_skip_broadcast;
    const bool use_s = (cfg.mac_mask & sm) && (!eth_addr || !l2skip || is_unicast_ethernet(s.srcaddr));
    const bool use_d = (cfg.mac_mask & dm) && (!eth_addr || !l2skip || is_unicast_ethernet(s.dstaddr));
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        sh[i] = use_s ? smac[i] : s.srcaddr[i];
        dh[i] = use_d ? dmac[i] : s.dstaddr[i];
    }
    if (c2s && !(cfg.mac_mask & dm)) {
        s.dst_modified = old_nz;
        pk.q18ev = (u8)((pk.q18ev & 4u) | 2u | (old_nz ? 1u : 0u));
    }
    en10mb_mac_rules(cfg, dh, sh);
    if (newl2 == 14) st16(pk.d + 12, (u16)s.proto);  // :691-694
    // the VLAN fields of the decoder's extra (en10mb.c:696-732): zero (never set) but for the
    // Juniper decoder, whose inner frame's en10mb decode filled them -- so behind any other
    // decoder a pushed tag's {TCI, inner type} land at byte 0, over the destination address,
    // and the inner type is the context's never-set proto_vlan_tag: 0
    if (cfg.vlan == TE_VLAN_ADD || (cfg.vlan == TE_VLAN_OFF && s.vlan)) {
        if ((int)s.vlan_offset + (cfg.vlan == TE_VLAN_ADD ? 4 : 2) > pktlen) {
            stale(pk, (int)NEED_NEVER);  // (past the new frame: the static buffer)
        } else {
            u8 *vh = pk.d + s.vlan_offset;
            if (cfg.vlan == TE_VLAN_ADD) {
                st16(pk.d + 12, bswap16((u16)cfg.vlan_proto));
                st16(vh + 2, bswap16((u16)s.proto_vlan_tag));
            }
            if (cfg.vlan_tag < 65535) st16(vh, bswap16((u16)cfg.vlan_tag & 0x0fff));
            else if (s.vlan) st16(vh, bswap16(s.vlan_tag));
            if (cfg.vlan_pri < 255) st16(vh, (u16)(ld16(vh) + bswap16((u16)(cfg.vlan_pri << 13))));
            else if (s.vlan) st16(vh, (u16)(ld16(vh) + bswap16(s.vlan_pri)));
            if (cfg.vlan_cfi < 255) st16(vh, (u16)(ld16(vh) + bswap16((u16)(cfg.vlan_cfi << 12))));
            else if (s.vlan) st16(vh, (u16)(ld16(vh) + bswap16(s.vlan_cfi)));
        }
    } else if (cfg.vlan == TE_VLAN_DEL) {
        st16(pk.d + 12, bswap16((u16)s.vlan_proto));  // htons(extra->vlan_proto)
    }
    return pktlen;
}

// Returns the new packet length (or RC_ERROR).  May move the packet start
// (pk.d) by -4 (VLAN push) / +4 (VLAN pop) together with its record header.
DI int en10mb_encode(Pkt &pk, const te_dev_cfg_t &cfg, Dec &s, int pktlen, int dir) {
    if (pktlen < 14) return RC_ERROR;
    if (cfg.vlan == TE_VLAN_ADD && !s.vlan && cfg.vlan_tag == 65535) return RC_ERROR;
    u32 newl2 = 0, oldl2 = 0;
    if (cfg.vlan == TE_VLAN_ADD) {
        oldl2 = s.vlan_offset;
        newl2 = s.vlan_offset + 4;
    } else if (cfg.vlan == TE_VLAN_DEL) {
        if (s.vlan) { oldl2 = s.vlan_offset + 4; newl2 = s.vlan_offset; }
    } else {
        if (s.vlan) { oldl2 = s.vlan_offset; newl2 = s.vlan_offset; }
    }
    if ((u32)pktlen < newl2 || pktlen + newl2 - s.l2len > MAXPACKET) return RC_ERROR;
    if (pktlen < s.l2len) return RC_ERROR;
    if (newl2 > 0 && newl2 != oldl2) {
        if (pktlen + (newl2 - oldl2) > MAXPACKET) return RC_ERROR;
        if (dir != TE_DIR_C2S && dir != TE_DIR_S2C) return RC_ERROR;  // checked below in the reference
        // move the record header + the first oldl2 bytes instead of the tail
        u8 *const old_d = pk.d;
        const u32 old_phys = pk.phys;
        if (newl2 > oldl2) {  // push 4 bytes at oldl2
            if (pk.room < 4) {  // no headroom left: flagged, never written past the slot
                stale(pk, (int)NEED_NEVER);
                return RC_ERROR;
            }
            pk.room -= 4;
            u8 *src = pk.d - 16, *dst = pk.d - 20;
            for (u32 i = 0; i < 16 + oldl2; ++i) dst[i] = src[i];
            pk.d -= 4;
        } else {  // pop 4 bytes at newl2
            u8 *src = pk.d - 16, *dst = pk.d - 12;
            for (int i = (int)(16 + newl2) - 1; i >= 0; --i) dst[i] = src[i];
            pk.d += 4;
            pk.avail -= 4;
            pk.phys -= 4;
            pk.room += 4;
        }
        // the reference's memmove (en10mb.c:568-578) writes its buffer up to pktlen +- 4
        pk.ext = (u32)(pktlen + (int)(newl2 - oldl2));
        if (pk.strict) {
            pk.phys = old_phys;
            strict_tail(pk, old_d);
        }
        if (newl2 > oldl2) {
            pk.avail += 4;
            pk.phys += 4;
        }
    }
    pktlen += (int)(newl2 - oldl2);
    u8 *eth = pk.d + s.l2offset;
    u8 *dh = eth, *sh = eth + 6;
    const bool l2skip = cfg.l2_skip_broadcast;
    if (dir == TE_DIR_C2S || dir == TE_DIR_S2C) {
        const bool c2s = dir == TE_DIR_C2S;
        const int sm = c2s ? TE_MASK_SMAC1 : TE_MASK_SMAC2, dm = c2s ? TE_MASK_DMAC1 : TE_MASK_DMAC2;
        const u8 *smac = c2s ? cfg.intf1_smac : cfg.intf2_smac;
        const u8 *dmac = c2s ? cfg.intf1_dmac : cfg.intf2_dmac;
        const bool use_s = (cfg.mac_mask & sm) && (!l2skip || is_unicast_ethernet(s.srcaddr));
        const bool use_d = (cfg.mac_mask & dm) && (!l2skip || is_unicast_ethernet(s.dstaddr));
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            sh[i] = use_s ? smac[i] : s.srcaddr[i];
            dh[i] = use_d ? dmac[i] : s.dstaddr[i];
        }
    } else {
        return RC_ERROR;
    }
    en10mb_mac_rules(cfg, dh, sh);
    if (newl2 == 14) st16(eth + 12, (u16)s.proto);
    if (cfg.vlan == TE_VLAN_ADD || (cfg.vlan == TE_VLAN_OFF && s.vlan)) {
        u8 *vh = pk.d + s.vlan_offset;  // {tci, tpid}
        if (cfg.vlan == TE_VLAN_ADD) {
            st16(pk.d + s.l2offset + 12, bswap16((u16)cfg.vlan_proto));
            st16(vh + 2, bswap16((u16)s.proto_vlan_tag));
        }
        if (cfg.vlan_tag < 65535) st16(vh, bswap16((u16)(cfg.vlan_tag & 0x0fff)));
        else if (s.vlan) st16(vh, bswap16(s.vlan_tag));
        if (cfg.vlan_pri < 255) st16(vh, (u16)(ld16(vh) + bswap16((u16)(cfg.vlan_pri << 13))));
        else if (s.vlan) st16(vh, (u16)(ld16(vh) + bswap16(s.vlan_pri)));
        if (cfg.vlan_cfi < 255) st16(vh, (u16)(ld16(vh) + bswap16((u16)(cfg.vlan_cfi << 12))));
        else if (s.vlan) st16(vh, (u16)(ld16(vh) + bswap16(s.vlan_cfi)));
    } else if (cfg.vlan == TE_VLAN_DEL && newl2 > 0) {
        st16(eth + 12, bswap16(s.vlan_proto));
    }
    return pktlen;
}

// Replace a decoded L2 header of s.l2len bytes by n new ones (dlt_user_encode's and
// dlt_hdlc_encode's memmove, user.c:245-253, hdlc.c:239-247): the payload stays where
// it is and the record's 16-byte pcap header moves, as the VLAN push/pop does above.
// A longer header moves into the slot's headroom (pk.room: what earlier moves of this
// record -- a first encode before a fuzz step's second one -- left of it); more than that
// is flagged unsupported.  The caller writes the n header bytes at the new pk.d.
DI bool l2_replace(Pkt &pk, int l2len, int n) {
    const int delta = l2len - n;
    if (delta == 0) return true;
    if (-delta > (int)pk.room) {
        stale(pk, (int)NEED_NEVER);  // slot headroom, not stale bytes: not replayed
        return false;
    }
    u8 *src = pk.d - 16, *dst = pk.d - 16 + delta;
    if (delta > 0)
        for (int i = 15; i >= 0; --i) dst[i] = src[i];
    else
        for (int i = 0; i < 16; ++i) dst[i] = src[i];
    u8 *const old_d = pk.d;
    const u32 old_phys = pk.phys;
    pk.d += delta;
    pk.avail -= delta;
    pk.phys -= delta;
    pk.room = (u32)((int)pk.room + delta);
    pk.ext = (u32)((int)pk.caplen - delta);  // user.c:245-253 / hdlc.c:239-247 memmove extent
    if (pk.strict) {
        pk.phys = old_phys;
        strict_tail(pk, old_d);
    }
    return true;
}

// dlt_user_encode (plugins/dlt_user/user.c:223-268): the --user-dlink bytes of the direction
DI int user_encode(Pkt &pk, const te_dev_cfg_t &cfg, const Dec &s, int pktlen, int dir) {
    if (pktlen == 0) return RC_ERROR;
    if (dir != TE_DIR_C2S && dir != TE_DIR_S2C) return RC_ERROR;
    const int n = cfg.user_length;
    if (!l2_replace(pk, s.l2len, n)) return RC_ERROR;
    const u8 *src = dir == TE_DIR_C2S ? cfg.user_l2client : cfg.user_l2server;
    for (int i = 0; i < n; ++i) pk.d[i] = src[i];
    return pktlen + n - s.l2len;
}

// An encoder's memmove that a later step of the same encode fails (dlt_hdlc_encode,
// hdlc.c:240-248 then :276/:286; dlt_en10mb_encode from another DLT, en10mb.c:567-578 then
// :600/:617/:634/:650): the payload at byte oldl2 moved to byte newl2 in place, the caplen
// unchanged -- the soft error writes the record so (tcpedit.c:104-108).  A move to a later
// byte also pushes the payload's last newl2 - oldl2 bytes past the record, into the buffer
// (written where the slot has room: only a later stale read would see them).
DI void l2_half_move(Pkt &pk, int oldl2, int newl2, int pktlen) {
    u8 *d = pk.d;
    if (oldl2 > newl2) {
        for (int i = newl2; i < pktlen - oldl2 + newl2; ++i) d[i] = d[i + oldl2 - newl2];
    } else if (oldl2 < newl2) {
        const int sh = newl2 - oldl2, end = pktlen + sh <= (int)pk.avail ? pktlen + sh : pktlen;
        for (int i = end - 1; i >= newl2; --i) d[i] = d[i - sh];
        if (end > (int)pk.ext) pk.ext = (u32)end;
    }
}

// dlt_hdlc_encode (plugins/dlt_hdlc/hdlc.c:223-290): {address, control, protocol}.
// Without --hdlc-address / --hdlc-control a field comes from `extra->hdlc` (:273, :283),
// the first int of the context's decoded extra: the en10mb decoder's `vlan` flag (1 for a
// tagged frame, en10mb_types.h:30), 0 behind every other decoder (zeroed, never written
// there); a 0 fails the encode after the memmove (l2_half_move)
DI int hdlc_encode(Pkt &pk, const te_dev_cfg_t &cfg, const Dec &s, int pktlen) {
    if (pktlen < 4) return RC_ERROR;
    // :237-238: behind a whole Juniper inner decode the decoded extra is too small
    if (s.jsub) return RC_ERROR;
    const int fb = cfg.decoder == TE_DEC_EN10MB ? s.vlan : 0;
    const bool aok = cfg.hdlc_address < 65535 || fb, cok = cfg.hdlc_control < 65535 || fb;
    const int addr = cfg.hdlc_address < 65535 ? (int)(u8)cfg.hdlc_address : (int)(u8)fb;
    if (!aok || !cok) {  // (the address byte goes in before the control field fails)
        l2_half_move(pk, s.l2len, 4, pktlen);
        if (aok) pk.d[0] = (u8)addr;
        return RC_ERROR;
    }
    if (!l2_replace(pk, s.l2len, 4)) return RC_ERROR;
    pk.d[0] = (u8)addr;
    pk.d[1] = cfg.hdlc_control < 65535 ? (u8)cfg.hdlc_control : (u8)fb;
    st16(pk.d + 2, (u16)s.proto);  // hdlc->protocol = ctx->proto
    return pktlen + 4 - s.l2len;
}

// dlt_en10mb_merge_layer3 (en10mb.c:847-887): multicast destination MAC unless
// dst_modified (never set behind the en10mb decoder: a memcmp of untouched bytes, :614;
// behind a Linux cooked decoder, Q18).
DI void en10mb_merge_layer3(Pkt &pk, const Dec &s, const u8 *ip, const u8 *ip6) {
    int pktlen = (int)pk.caplen;
    int l2len = en10mb_l2len(pk.d, pktlen);
    if (l2len == -1 || pktlen < l2len) return;
    u8 *dh = pk.d + s.l2offset;
    if (ip) {
        if (pktlen >= 34 && !s.dst_modified) {
            u32 dst = ld32(ip + 16);
            if (mcast4(dst)) {
                u32 c = bswap32(dst);
                dh[0] = 0x01; dh[1] = 0x00; dh[2] = 0x5e;
                dh[3] = (u8)(c >> 16) & 0x7f; dh[4] = (u8)(c >> 8); dh[5] = (u8)c;
            }
        }
    } else if (ip6) {
        if (pktlen >= 54 && !s.dst_modified) {
            const u8 *a = ip6 + 24;
            if (a[0] == 0xff) {
                dh[0] = 0x33; dh[1] = 0x33; dh[2] = a[12]; dh[3] = a[13]; dh[4] = a[14]; dh[5] = a[15];
            }
        }
    }
}

// the encoder's L2 length (plugin_l2len): en10mb's parse (en10mb.c:917-943),
// user.c:325-342, hdlc.c:355-366
DI int encoder_l2len_d(const u8 *d, u32 caplen, const te_dev_cfg_t &cfg) {
    return cfg.encoder == TE_ENC_USER                                   ? cfg.user_length
           : (cfg.encoder == TE_ENC_HDLC || cfg.encoder == TE_ENC_PPP) ? (caplen < 4 ? -1 : 4)  // pppserial.c:335-343
                                                                       : en10mb_l2len(d, (int)caplen);
}
DI int encoder_l2len(const Pkt &pk, const te_dev_cfg_t &cfg) { return encoder_l2len_d(pk.d, pk.caplen, cfg); }

// ---------------------------------------------------------------------------
// --fuzz-seed: fuzzing() (src/tcpedit/fuzzing.c:62-297) for one packet.  The
// reference draws one tcpr_random() from a run-wide state per packet that
// reaches this step (tcpedit.c:250-258); the launch hands each such packet the
// state it would see, found by a reach pass, a prefix count and an LCG jump
// (te_fuzz_states).  Writes the reference makes past caplen (its l4len is an
// offset from the packet start, fuzzing.c:118,127) land in its static buffer and
// never reach the output: here they are kept only inside this lane's slot.
// ---------------------------------------------------------------------------
DI u32 tcpr_random_dev(u32 &seed) {  // utils.c:436-458
    u32 n = seed, r;
    n = n * 1103515245u + 12345u;
    r = (u32)((int)(n / 65536) % 2048);
    n = n * 1103515245u + 12345u;
    r = (r << 10) ^ (u32)((int)(n / 65536) % 1024);
    n = n * 1103515245u + 12345u;
    r = (r << 10) ^ (u32)((int)(n / 65536) % 1024);
    seed = n;
    return r;
}

DI u32 fuzz_sgt_size(u32 r, u32 caplen) {  // fuzzing.c:23-35
    return caplen == 0 ? 0u : caplen <= 16 ? 1u : 1u + r % 15u;
}

DI void fuzz_fill(Pkt &pk, int from, int n, int how, u8 x) {  // how: 0 = 0x00, 1 = 0xff, 2 = ^x
    for (int i = 0; i < n; ++i) {
        const int j = from + i;
        // past the lane's slot: the reference's stale buffer, never output.  A byte past
        // `phys` stays unknown here (an XOR of a stale byte), and any later read of one
        // is flagged where it happens.
        if (j < 0 || j >= (int)pk.avail) continue;
        if (how == 2 && pk.strict && j >= (int)pk.phys) stale(pk, j + 1);
        pk.d[j] = how == 0 ? (u8)0 : how == 1 ? (u8)0xff : (u8)(pk.d[j] ^ x);
        if ((u32)j >= pk.ext) pk.ext = (u32)j + 1;
    }
}

// What fuzzing() does to a record it picked (fuzzing.c:133-199), from the draw r and the
// payload's place (l4off = l4data - packet, l4len as the reference computes it): a size cut
// (DROP / REDUCE: caplen = len = nl) or a byte run [from, from + n) set to 0x00 / 0xff or
// XORed with x (how 0 / 1 / 2), and fuzzing()'s return (chksum_update_required).  Reads
// nothing: the wave lane plans its records with it, and fuzz_plan below the others.
struct FzPlan {
    int ret = 0;
    bool cut = false;
    u32 nl = 0;
    int from = 0, n = 0, how = 0;
    u8 x = 0;
    int stale_at = 0;  // > 0: the IP protocol byte was read at or past `phys` (fuzz_plan)
};
DI FzPlan fuzz_plan_l4(u32 r, int l4off, int l4len, u32 caplen, u32 len) {
    FzPlan f;
    if (l4len <= 1 || l4off > (int)caplen) return f;
    r ^= r >> 16;
    const u32 act = r % 11u;  // fuzzing.h: DROP, REDUCE, START_{0,R,FF}, MID_{0,R,FF}, END_{0,R,FF}
    f.x = (u8)(r >> 4);
    if (act <= 1) {  // fuzz_reduce_packet_size (fuzzing.c:37-60): DROP returns 0, REDUCE 1
        const u32 nl = act == 0 ? 0u : r % (u32)(l4len - 1) + 1u;
        if (len < caplen || nl > caplen) return f;
        f.ret = (int)act;
        f.cut = nl != caplen;
        f.nl = nl;
        return f;
    }
    if (act <= 4) {  // START_*
        const int sgt = (int)fuzz_sgt_size(r, (u32)l4len);
        if (!sgt && act != 2) return f;
        f.from = l4off;
        f.n = sgt;
        f.how = act == 2 ? 0 : act == 4 ? 1 : 2;
        f.ret = 1;
        return f;
    }
    if (act <= 7) {  // MID_*
        if (act != 6 && l4len <= 2) return f;
        const u32 off = ((r >> 16) % (u32)(l4len - 1)) + 1u;
        const int sgt = (int)fuzz_sgt_size(r, (u32)l4len - off);
        if (!sgt || (act == 6 && sgt > l4len)) return f;
        f.from = l4off + (int)off;
        f.n = sgt;
        f.how = act == 5 ? 0 : act == 7 ? 1 : 2;
        f.ret = 1;
        return f;
    }
    const int sgt = (int)fuzz_sgt_size(r, (u32)l4len);  // END_*
    if (!sgt || sgt > l4len) return f;
    f.from = l4off + l4len - sgt;
    f.n = sgt;
    f.how = act == 8 ? 0 : act == 10 ? 1 : 2;
    f.ret = 1;
    return f;
}

// fuzzing() for a picked record d[0, caplen) as the encoder left it (fuzzing.c:89-131:
// the encoder's l2len and protocol, the L4 header's place); `phys`: the bytes from d
// that are the record's (a read past them is a stale static-buffer read, Q8)
DI FzPlan fuzz_plan(const u8 *d, u32 caplen_u, u32 len, u32 phys, const te_dev_cfg_t &cfg, u32 r) {
    const int caplen = (int)caplen_u;
    const int l2len = encoder_l2len_d(d, caplen_u, cfg);
    int proto = -1;  // plugin_proto: en10mb.c:741-762, user.c:271-279 (always an error), hdlc.c:300-312
    if (cfg.encoder == TE_ENC_HDLC) {
        if (caplen >= 4) proto = ld16(d + 2);
    } else if (cfg.encoder == TE_ENC_EN10MB && caplen >= 14) {
        L2 q;
        if (get_l2len_protocol(d, caplen_u, q) != -1) proto = bswap16(q.protocol);
    }
    const u16 l2proto = bswap16((u16)proto);
    if (l2len == -1 || caplen < l2len || caplen <= l2len) return FzPlan{};  // :95-109, dlt_utils.c:195
    int l4off, l4len;  // l4data - packet, and the reference's l4len
    u8 l4proto;
    int stale_at = 0;
    if (l2proto == 0x0800 || l2proto == 0x86DD) {
        const u8 *ip = d + l2len;
        const bool v4 = l2proto == 0x0800;
        const int l4 = v4 ? l4_v4(ip, caplen - l2len) : l4_v6(ip, 0, caplen - l2len);
        if (l4 < 0) return FzPlan{};
        l4off = l2len + l4;
        l4len = l4off;  // an offset, as the reference has it (fuzzing.c:118,127)
        const int pb = l2len + (v4 ? 9 : 6);
        if (pb >= (int)phys) stale_at = pb + 1;
        l4proto = ip[v4 ? 9 : 6];
    } else {
        l4len = caplen - l2len;
        l4off = l2len;
        l4proto = 255;
    }
    if (l4proto == 6) {
        l4len -= 20;
        l4off += 20;
    } else if (l4proto == 17) {
        l4len -= 8;
        l4off += 8;
    }
    FzPlan f = fuzz_plan_l4(r, l4off, l4len, caplen_u, len);
    f.stale_at = stale_at;
    return f;
}

DI int fuzz_packet(Pkt &pk, const te_dev_cfg_t &cfg, u32 state) {
    const u32 r = tcpr_random_dev(state);
    if (r % cfg.fuzz_factor) return 0;
    const FzPlan f = fuzz_plan(pk.d, pk.caplen, pk.len, pk.phys, cfg, r);
    if (f.stale_at) stale(pk, f.stale_at);
    if (f.cut) pk.len = pk.caplen = f.nl;
    if (f.n) fuzz_fill(pk, f.from, f.n, f.how, f.x);
    return f.ret;
}

// ---------------------------------------------------------------------------
// tcpedit_packet (src/tcpedit/tcpedit.c:46-366).
// Returns RC_* ; *warned set when the checksum step warned (:351-353).
// fz_mode: TE_FUZZ_OFF; TE_FUZZ_PROBE returns RC_REACHED at the fuzz step (the
// reach pass); TE_FUZZ_APPLY fuzzes with RNG state fz_state there.
// ---------------------------------------------------------------------------
constexpr int RC_REACHED = 3;
// ANYDEC: the instance for the other decoders and encoders (cfg.decoder != EN10MB, or a
// non-encoding / pppserial encoder); without it those paths are compiled out, so the
// Ethernet edit keeps its register budget.
template <bool FZ = false, bool ANYDEC = false>
DI int tcpedit_packet(Pkt &pk, const te_dev_cfg_t &cfg, const u16 *portlut, int dir, bool &warned,
                      u32 fz_mode = TE_FUZZ_OFF, u32 fz_state = 0) {
    warned = false;
    u8 *ip = nullptr, *ip6 = nullptr;
    int needtorecalc = 0, retval = 0;

    if (cfg.efcs && pk.len > 4) {  // :78-84
        if (pk.caplen == pk.len) pk.caplen -= 4;
        pk.len -= 4;
    }
    bool fuzz_once = FZ && fz_mode != TE_FUZZ_OFF;  // :49
    int l2proto, l2len, l3len;
    Dec s;
again:  // :89 -- after the fuzz step the packet goes through L2 and the L3 edits once more
    ip = ip6 = nullptr;
    retval = 0;
    // l2proto (:96): the decoder's proto, network-order value
    if constexpr (ANYDEC) {
        l2proto = decoder_proto(pk, cfg);
    } else {  // dlt_en10mb_proto (en10mb.c:741-762)
        L2 r;
        l2proto = pk.caplen < 14 || get_l2len_protocol(pk.d, pk.caplen, r) == -1 ? RC_ERROR : bswap16(r.protocol);
    }
    if (l2proto < 0) return RC_SOFT;
    s.dst_modified = pk.l2carry != 0;
    // tcpedit_dlt_process (dlt_plugins.c:210-238)
    int pktlen;
    if (dir == TE_DIR_NOSEND) {
        pktlen = (int)pk.caplen;
        s.l2offset = 0;
    } else {
        if constexpr (FZ && ANYDEC) {
            // the second decode of a fuzzed record (tcpedit.c:89,250-258) by the Juniper
            // decoder: a warning frame reads the state this record's first pass left (its own
            // whole decode, else the carried one: the scan's next entry); a whole decode
            // would write state the scan did not see -- not served (fails loudly)
            u32 hl = 0;
            if (cfg.decoder == TE_DEC_JNPR && fz_mode == TE_FUZZ_APPLY && !fuzz_once) {
                pk.jc = pk.jc2;
                pk.jnone = pk.jnone2;
                if (jnpr_header(pk.d, pk.caplen, hl) == RC_OK) {
                    stale(pk, (int)NEED_NEVER);
                    return RC_SOFT;
                }
            }
        }
        if ((ANYDEC && cfg.decoder != TE_DEC_EN10MB ? foreign_decode(pk, cfg, s)
                                                    : en10mb_decode(pk.d, (int)pk.caplen, s)) == RC_ERROR)
            return RC_SOFT;
        if (cfg.encoder == TE_ENC_USER)
            pktlen = user_encode(pk, cfg, s, (int)pk.caplen, dir);
        else if (cfg.encoder == TE_ENC_HDLC)
            pktlen = hdlc_encode(pk, cfg, s, (int)pk.caplen);
        else if (ANYDEC && cfg.encoder == TE_ENC_NOENC)  // linuxsll.c:201-208 and the like
            pktlen = RC_ERROR;
        else if (ANYDEC && cfg.encoder == TE_ENC_PPP)  // pppserial.c:239-251
            pktlen = pk.caplen < 4 ? RC_ERROR : (int)pk.caplen;
        else if (ANYDEC && cfg.decoder != TE_DEC_EN10MB)
            pktlen = en10mb_encode_foreign(pk, cfg, s, (int)pk.caplen, dir);
        else
            pktlen = en10mb_encode(pk, cfg, s, (int)pk.caplen, dir);
        if (pktlen < 0) return RC_SOFT;
    }
    int lendiff = pktlen - (int)pk.caplen;  // :111-113
    pk.caplen += lendiff;
    pk.len += lendiff;

    l2len = encoder_l2len(pk, cfg);  // :116
    if (l2len == -1) return RC_SOFT;

    if (l2proto == 0x0008) {  // htons(ETHERTYPE_IP)  :123-148
        if (pk.caplen < (u32)l2len + 20) return RC_SOFT;
        if ((int)pk.caplen <= l2len) return RC_SOFT;  // tcpedit_dlt_l3data_copy (dlt_utils.c:195)
        ip = pk.d + l2len;
        if (l4_v4(ip, (int)pk.caplen - l2len) < 0) return RC_SOFT;
    } else if (l2proto == 0xDD86) {  // htons(ETHERTYPE_IP6)  :149-173
        if (pk.caplen < (u32)l2len + 40) return RC_SOFT;
        if ((int)pk.caplen <= l2len) return RC_SOFT;
        ip6 = pk.d + l2len;
        if (l4_v6(ip6, 0, (int)pk.caplen - l2len) < 0) return RC_SOFT;
    }

    l3len = (int)pk.caplen - l2len;
    if (ip) {  // :182-206
        if (cfg.tos > -1) {
            u16 oldv = ld16(ip);
            u16 newv = bswap16((u16)((bswap16(oldv) & 0xff00) | (cfg.tos & 0xff)));
            st16(ip, newv);
            csum_replace2(ip + 10, oldv, newv);
        }
        if (cfg.ttl_mode != TE_TTL_OFF) {  // rewrite_ipv4_ttl (edit_packet.c:627-667)
            u8 t = ip[8], v = (u8)cfg.ttl_value;
            bool changed = true;
            if (cfg.ttl_mode == TE_TTL_SET) {
                if (t == v) changed = false;
                else t = v;
            } else if (cfg.ttl_mode == TE_TTL_ADD) {
                t = ((int)t + v > 255) ? 255 : (u8)(t + v);
            } else {
                t = (t <= v) ? 1 : (u8)(t - v);
            }
            if (changed) {
                u16 oldv = ip[8];
                ip[8] = t;
                csum_replace2(ip + 10, oldv, (u16)t);
                needtorecalc += 1;
            }
        }
        if (cfg.has_portmap) {  // rewrite_ipv4_ports (portmap.c:332-351)
            if (ip[9] == 6 || ip[9] == 17) {
                int l4 = l4_v4(ip, l3len);
                retval = l4 >= 0 ? rewrite_ports(portlut, ip[9], ip + l4, l3len - l4) : RC_WARN;
            } else {
                retval = 0;
            }
            needtorecalc += retval;
        }
        if (cfg.tcp_sequence_enable && ip[9] == 6) {  // rewrite_sequence.c:57-74
            int l4 = l4_v4(ip, l3len);
            if (l4 >= 0) rewrite_seqs(pk, cfg, ip + l4);
        }
    } else if (ip6) {  // :209-248
        if (cfg.ttl_mode != TE_TTL_OFF) {  // rewrite_ipv6_hlim (edit_packet.c:673-706)
            u8 t = ip6[7], v = (u8)cfg.ttl_value;
            bool changed = true;
            if (cfg.ttl_mode == TE_TTL_SET) {
                if (t == v) changed = false;
                else t = v;
            } else if (cfg.ttl_mode == TE_TTL_ADD) {
                t = ((int)t + v > 255) ? 255 : (u8)(t + v);
            } else {
                t = (t <= v) ? 1 : (u8)(t - v);
            }
            ip6[7] = t;
            needtorecalc += changed ? 1 : 0;
        }
        if (cfg.tclass > -1) {
            u32 f = (be32(ip6) & 0xf00fffffu) + ((u32)cfg.tclass << 20);
            st32(ip6, bswap32(f));
        }
        if (cfg.flowlabel > -1) {
            u32 f = (be32(ip6) & 0xfff00000u) + (u32)cfg.flowlabel;
            st32(ip6, bswap32(f));
        }
        if (cfg.has_portmap) {  // rewrite_ipv6_ports (portmap.c:353-372)
            if (ip6[6] == 6 || ip6[6] == 17) {
                int l4 = l4_v6(ip6, 0, l3len);
                retval = l4 >= 0 ? rewrite_ports(portlut, ip6[6], ip6 + l4, l3len - l4) : RC_WARN;
            } else {
                retval = 0;
            }
            needtorecalc += retval;
        }
        if (cfg.tcp_sequence_enable && ip6[6] == 6) {  // rewrite_sequence.c:76-92
            int l4 = l4_v6(ip6, 0, l3len);
            if (l4 >= 0) rewrite_seqs(pk, cfg, ip6 + l4);
        }
    }

    if constexpr (FZ) {
        if (fuzz_once) {  // :250-258
            if (fz_mode == TE_FUZZ_PROBE) return RC_REACHED;
            fuzz_once = false;
            retval = fuzz_packet(pk, cfg, fz_state);
            needtorecalc += retval;
            pk.q18ev |= 4u;
            goto again;
        }
    }

    if (cfg.fixlen || cfg.mtu_truncate) {  // :261-265
        retval = untrunc_packet(pk, cfg, ip, ip6);
        if (retval < 0) return RC_ERROR;
        needtorecalc += retval;
    }

    l3len = (int)pk.caplen - l2len;
    if (cfg.rewrite_ip) {  // :268-290
        if (ip) {
            rewrite_ipv4l3(cfg, ip, dir, l3len);
            retval = 0;
        } else if (ip6) {
            rewrite_ipv6l3(pk, cfg, ip6, dir, l3len);
            retval = 0;
        } else if (l2proto == 0x0608) {
            rewrite_iparp(pk, cfg, pk.d + l2len, dir);
        }
    }

    if (cfg.seed) {  // :293-317
        if (ip) {  // randomize_ipv4 (edit_packet.c:420-467)
            if (l3len < (int)(ip[0] & 0x0f) << 2) return RC_ERROR;
            if (!(cfg.skip_broadcast && mcast4(ld32(ip + 16)))) {
                u32 o = ld32(ip + 16);
                st32(ip + 16, randomize_ipv4_addr(cfg, o));
                ipv4_addr_csum_replace(ip, o, ld32(ip + 16), l3len);
            }
            if (!(cfg.skip_broadcast && mcast4(ld32(ip + 12)))) {
                u32 o = ld32(ip + 12);
                st32(ip + 12, randomize_ipv4_addr(cfg, o));
                ipv4_addr_csum_replace(ip, o, ld32(ip + 12), l3len);
            }
            retval = 0;
        } else if (ip6) {  // randomize_ipv6 (edit_packet.c:469-518)
            if (l3len < 40) return RC_ERROR;
#pragma unroll
            for (int which = 0; which < 2; ++which) {
                int ao = which == 0 ? 24 : 8;
                if (!(cfg.skip_broadcast && mcast6(ip6 + ao))) {
                    u8 old[16];
                    for (int b = 0; b < 16; ++b) old[b] = ip6[ao + b];
                    randomize_ipv6_addr(cfg, ip6 + ao);
                    ipv6_addr_csum_replace(pk, ip6, old, ip6 + ao, l3len);
                }
            }
            retval = 0;
        } else if (l2proto == 0x0608) {  // randomize_iparp (edit_packet.c:1025-1083)
            if (l3len < 8) return RC_ERROR;
            int al2 = get_l2len(pk.d, pk.caplen);
            u8 *ip1, *ip2;
            if (arp_addrs(pk, pk.d + al2, &ip1, &ip2)) {
                st32(ip1, randomize_ipv4_addr(cfg, ld32(ip1)));
                st32(ip2, randomize_ipv4_addr(cfg, ld32(ip2)));
            }
        }
    }

    if (cfg.fixhdrlen) {  // :321-335
        int changed = 0;
        if (ip) {  // fix_ipv4_length (edit_packet.c:381-396)
            if (pk.caplen < (u32)l2len + 20) {
                changed = -1;
            } else if ((be16(ip + 6) & 0x3fff) == 0 && (int)be16(ip + 2) != (int)(pk.len - (u32)l2len)) {
                st16(ip + 2, bswap16((u16)(pk.len - (u32)l2len)));
                changed = 1;
            }
        } else if (ip6) {  // fix_ipv6_length (edit_packet.c:398-413)
            int want = (int)(pk.len - (u32)l2len - 40);
            if (pk.caplen < (u32)l2len + 40) {
                changed = -1;
            } else if ((int)be16(ip6 + 4) != want) {
                st16(ip6 + 4, bswap16((u16)want));
                changed = 1;
            }
        }
        if (changed > 0) needtorecalc |= changed;
    }

    if (cfg.fixcsum || needtorecalc > 0) {  // :338-354
        if (ip) retval = fix_ipv4_checksums(pk, ip, l2len);
        else if (ip6) retval = fix_ipv6_checksums(pk, ip6, l2len);
        else retval = RC_OK;
        if (retval < 0) return RC_ERROR;
        if (retval == RC_WARN) warned = true;
    }

    // :356-361; the user and hdlc encoders merge in place (dlt_utils.c:189-221)
    if (cfg.encoder == TE_ENC_EN10MB) en10mb_merge_layer3(pk, s, ip, ip6);
    return retval;
}

}  // namespace te
