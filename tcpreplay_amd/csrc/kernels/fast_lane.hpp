// fast_lane.hpp -- register-resident tcpedit_packet for the dominant header shapes.
//
// One lane edits one packet whose headers are plain Ethernet II + IPv4 (IHL 5,
// not a fragment, ip_len == caplen - 14) or IPv6 (TCP/UDP directly after the
// fixed header, payload length == caplen - 54), TCP or UDP, caplen == len.
// With a 14-byte Ethernet header every IP/L4 field sits at a packet offset
// that is 2 mod 4, so the lane loads an 80-byte window aligned to packet offset
// -2 into 20 VGPRs:  H[i] = little-endian dword of packet bytes [4i-2, 4i+2).
// Every address, port and checksum word is then a whole dword or half-dword
// at a compile-time index, and every one's-complement word of the headers is a
// 16-bit half of some H[i] (relative offsets 4i-2 and 4i are even).
//
// The edits are the reference's, step for step, in tcpedit_packet's order
// (tcpedit.c:46-366): en10mb MAC rewrite (en10mb.c:479-736), port map
// (portmap.c:239-372), srcip/dstip/pnat/endpoint maps (edit_packet.c:787-1019),
// seed randomisation (:336-518), full checksums (:55-189, checksum.c:34-170),
// multicast destination MAC (en10mb.c:847-887).  They reuse edit_pkt.hpp's value
// helpers (randomize_ipv4_addr, remap_ipv4, ip_in_cidr, csum_replace*_v), so the
// two lanes share their arithmetic.  Only the UDP checksum field is carried
// through the incremental updates: with --fixcsum every other checksum is
// recomputed from scratch, but a UDP field the updates leave at 0 is NOT
// recomputed (checksum.c:115), so its incremental value decides.
//
// Whatever is not one of these shapes, or needs an option the fast lane does
// not carry (the host clears te_fast_cfg_t.ok), is deferred to the generic lane.
#pragma once
#include "edit_pkt.hpp"

namespace te {
namespace fl {

constexpr int NW = 20;            // window dwords
constexpr int WEND = 4 * NW - 2;  // 78: first packet byte past the window

DI u32 lo16(u32 x) { return x & 0xffffu; }
DI u32 hi16(u32 x) { return x >> 16; }
DI u32 with_lo16(u32 x, u32 v) { return (x & 0xffff0000u) | (v & 0xffffu); }
DI u32 with_hi16(u32 x, u32 v) { return (x & 0xffffu) | (v << 16); }
DI u32 wsum(u32 x) { return (x & 0xffffu) + (x >> 16); }  // its two LE 16-bit words
// acc + the two LE 16-bit words of x, in one v_sad_u16 (|x.lo - 0| + |x.hi - 0| + acc)
DI u32 wsum_acc(u32 x, u32 acc) { return __builtin_amdgcn_sad_u16(x, 0u, acc); }
DI u32 swap16(u32 x) {
    x &= 0xffffu;  // (u16) truncation first, as bswap16((u16)...)
    return ((x >> 8) | (x << 8)) & 0xffffu;
}
DI u32 bs16(u32 x) { return swap16(x); }
// end-around-carry fold of a sum below 2^32 to 16 bits: two steps always suffice
// (fold16's data-dependent loop, unrolled for this range)
DI u32 fold32(u32 x) {
    x = (x & 0xffffu) + (x >> 16);
    return (x & 0xffffu) + (x >> 16);
}

// mask of bytes [lo, hi) of a dword (lo, hi clamped to [0, 4])
DI u32 bmask(int lo, int hi) {
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    const u32 mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
    const u32 ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
    return mh & ~ml;
}

// a[min(k, 3)] by masks: a ternary chain on a lane-varying k becomes a dynamically
// indexed stack array
DI u32 sel4(const u32 *a, u32 k) {
    return (a[0] & (0u - (u32)(k == 0))) | (a[1] & (0u - (u32)(k == 1))) | (a[2] & (0u - (u32)(k == 2))) |
           (a[3] & (0u - (u32)(k >= 3)));
}

// ip6_in_cidr (cidr.c:478-529) on an address held as 4 LE dwords, as one expression
// (a /0 mask matches every address there, zero or not)
DI bool ip6_in_cidr_w(const te_cidr_t &c, const u32 *a) {
    const int j = c.masklen / 8, r = c.masklen % 8;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) ok &= ((a[k] ^ ld32(c.network6 + 4 * k)) & bmask(0, j - 4 * k)) == 0;
    const u32 km = (0xffu << (8 - r)) & 0xffu;
    const u32 ab = (sel4(a, (u32)j >> 2) >> (8 * (j & 3))) & 0xffu;
    const bool last = r == 0 || (ab & km) == (c.network6[j & 15] & km);
    return (c.family == 6) & ok & last;
}

// ip_in_cidr (cidr.c:425-468) as one expression (64-bit mask semantics)
DI bool ip_in_cidr_f(const te_cidr_t &c, u32 ip_le) {
    const unsigned long long mask = ~0ull << (32 - c.masklen);
    const bool in = (((unsigned long long)bswap32(ip_le)) & mask) == (((unsigned long long)bswap32(c.network)) & mask);
    return (c.family == 4) & (in | ((c.masklen == 0) & (c.network == 0)));
}

// randomize_ipv6_addr (edit_packet.c:359-379); s = bswap32(seed)
DI void randomize_ipv6_w(u32 s, u32 *a) {
    const bool was = (a[0] & 0xffu) == 0xffu;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = (a[i] ^ s) - (a[i] & s);
    const bool now = (a[0] & 0xffu) == 0xffu;
    if (was && !now) a[0] = (a[0] & ~0xffu) | 0xffu;
    else if (!was && now) a[0] = (a[0] & ~0xffu) | 0xaau;
}

// is_unicast_ethernet (plugins/ethernet.c:30-57) on a MAC in the low 48 bits
DI bool unicast48(unsigned long long m) {
    if ((m & 0xffffffffffffull) == 0xffffffffffffull) return false;
    if ((m & 0xffffffull) == 0x5e0001ull) return false;  // 01:00:5e
    if ((m & 0xffffull) == 0x3333ull) return false;      // 33:33
    if ((m & 0xffffffffull) == 0x00500000ull && (((m >> 32) & 0xff) == 1 || ((m >> 32) & 0xff) == 2))
        return false;  // 00:00:50:00:01/02 (defines.h.in:226-227)
    return true;
}
DI unsigned long long mac48(const u8 *m) {
    return (unsigned long long)ld32(m) | ((unsigned long long)ld16(m + 4) << 32);
}

// Feature instances: F (TE_FF_* bits) names the option groups a kernel
// instance compiles in; a group left out is dead code, not a runtime branch on
// an LDS cfg field.  The host launches the smallest instance whose F covers the
// config (te_launch_edit).
constexpr u32 F_MAC = TE_FF_MAC, F_PORTMAP = TE_FF_PORTMAP, F_RWIP = TE_FF_RWIP, F_SEED = TE_FF_SEED;
constexpr u32 F_HDR = TE_FF_HDR, F_INCR = TE_FF_INCR;

// the scalar options phase A reads per packet, held in SGPRs (kernel arguments)
// instead of being re-read from the LDS cfg copy on every tile
struct Knobs {
    u32 seed_sw;      // bswap32(cfg.seed), as randomize_ipv4/6 use it
    bool seed;        // cfg.seed != 0
    bool skip_bcast;  // cfg.skip_broadcast
};
DI Knobs knobs_of(const te_dev_cfg_t &cfg) { return Knobs{bswap32(cfg.seed), cfg.seed != 0, cfg.skip_broadcast != 0}; }

// remap_ipv6 (edit_packet.c:748-779) for octet masks (the host keeps the
// non-octet out-of-range write of SURVEY Q9 on the generic lane)
DI void remap_ipv6_w(const Knobs &kn, const te_cidr_t &c, u32 *a) {
    const bool skip = (c.family != 6) | (kn.skip_bcast & ((a[0] & 0xffu) == 0xffu));
    const int j = c.masklen / 8;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32 m = skip ? 0u : bmask(0, j - 4 * k);
        a[k] = (a[k] & ~m) | (ld32(c.network6 + 4 * k) & m);
    }
}

// remap_ipv4 (edit_packet.c:713-746) as one expression; x86 masks a shift by 32 to 0
DI u32 remap_ipv4_f(const Knobs &kn, const te_cidr_t &c, u32 orig) {
    u32 mask = 0xffffffffu << ((32 - c.masklen) & 31);
    const u32 network = bswap32(c.network) & mask;
    mask ^= 0xffffffffu;
    const u32 r = bswap32(network ^ (bswap32(orig) & mask));
    return c.family != 4 ? 0u : ((kn.skip_bcast && mcast4(orig)) ? orig : r);
}

// what phase B needs to finish a packet after the block's chunk-prefix pass
struct State {
    u32 l4sum;  // unfolded one's-complement sum so far (pseudo header + L4 bytes inside the window)
    u32 end;    // caplen: L4 bytes run to here
    u32 dirty;  // bit i: H[i] may differ from the packet bytes (written back)
    bool v6, tcp, do_l4, tail;
};

// ---------------------------------------------------------------------------
// Phase A: classify, edit, IPv4 header checksum, in-window L4 sum.
// Returns false to defer the packet to the generic lane.
//
// The body has no lane-divergent control flow.  Every lane runs the same
// instructions and takes its results by selects; the option blocks and the
// IPv4 / IPv6 address blocks branch only on wave-uniform conditions (cfg fields,
// ballots).  A lane whose packet is deferred or not edited computes values that
// are never used: its tile goes to the generic lane, or its H is not written
// back.  (Divergent branches around edits of H made the compiler copy the whole
// window between register sets at every merge.)
//
// `part`: the window's one partly valid dword (packet bytes [4k - 2, caplen) with
// k = (caplen + 2) / 4 < NW, the rest zeroed; 0 when there is none), which the
// caller reads from the unedited image.  It is always L4 payload: a packet on
// this lane has its whole L4 header inside caplen, and the header dwords are whole.
//
// `tcap` (--mtu-trunc, SZ_MTU instances; 0 otherwise): the packet is classified with its
// captured caplen/len, then cut to tcap = 14 + mtu bytes as untrunc_packet does
// (edit_packet.c:596-611, after the header edits and before the address edits, tcpedit.c:
// 261-265): caplen = len = tcap, IPv4 total length = mtu, IPv6 payload length = mtu - 40,
// and the checksums cover the cut packet.  `part` is then the cut packet's.
//
// `force` (SZ_FUZZ instances): fuzzing() changed the packet (its 1 is a needtorecalc,
// tcpedit.c:252-256), so an F_INCR run checksums it from scratch too.
// ---------------------------------------------------------------------------
template <u32 F>
DI bool phase_a(u32 (&H)[NW], u32 caplen, u32 len, u32 part, int dir, const te_dev_cfg_t &cfg, const Knobs &kn,
                bool v6_ok, const TE_AS_GLOBAL uint16_t *lut, State &st, u32 tcap = 0, bool force = false) {
    // ---- classify: Ethernet II + IPv4 (IHL 5, no fragment, ip_len == caplen - 14) or
    // IPv6 (payload length == caplen - 54), then TCP or UDP with a whole header ----
    const u32 et = hi16(H[3]);  // bytes 12,13 as a raw LE u16
    const u32 ip_len = bs16(hi16(H[4]));
    const bool ok4 = (et == 0x0008u) & ((H[4] & 0xffu) == 0x45u) & (ip_len == caplen - 14) &  // Q4 warning path
                     (ip_len >= 20) & ((bs16(hi16(H[5])) & 0x3fffu) == 0);                    // and fragments: generic
    const u32 plen_raw = lo16(H[5]), l4len6 = bs16(plen_raw);
    const bool v6 = et == 0xDD86u;  // ETHERTYPE_IP6
    // (--mtu-trunc: edit_packet.c:167 sees the cut packet's payload length)
    const u32 plen_chk = tcap != 0 ? bs16(tcap - 54u) : plen_raw;
    const bool ok6 = v6 & v6_ok & (((H[4] >> 4) & 0xfu) == 6u) & (caplen >= 54) & (l4len6 == caplen - 54) &
                     !((caplen > 56) & (plen_chk < 40));  // raw network-order compare (edit_packet.c:167)
    const u32 proto = v6 ? (H[5] >> 16) & 0xffu : (H[6] >> 8) & 0xffu;
    const bool cut = tcap != 0;
    const u32 l4len = cut ? tcap - (v6 ? 54u : 34u) : (v6 ? l4len6 : ip_len - 20);
    const bool tcp = proto == 6;
    const bool ok = (caplen == len) & ((dir == TE_DIR_C2S) | (dir == TE_DIR_S2C)) & (ok4 | ok6) &
                    (tcp ? l4len >= 20 : ((proto == 17) & (l4len >= 8)));
    const bool c2s = dir == TE_DIR_C2S;

    u32 dirty = 0;
    // ---- en10mb_encode: MAC rewrite, then --enet-subsmac and --enet-mac-seed over the new
    // addresses (en10mb.c:586-689; en10mb_mac_rules) ----
    if ((F & F_MAC) && (cfg.mac_mask || cfg.n_subs || cfg.random_set)) {
        const int sm = c2s ? TE_MASK_SMAC1 : TE_MASK_SMAC2, dm = c2s ? TE_MASK_DMAC1 : TE_MASK_DMAC2;
        unsigned long long dmac = (unsigned long long)hi16(H[0]) | ((unsigned long long)H[1] << 16);
        unsigned long long smac = (unsigned long long)H[2] | ((unsigned long long)lo16(H[3]) << 32);
        const bool use_s = (cfg.mac_mask & sm) && (!cfg.l2_skip_broadcast || unicast48(smac));
        const bool use_d = (cfg.mac_mask & dm) && (!cfg.l2_skip_broadcast || unicast48(dmac));
        smac = use_s ? mac48(c2s ? cfg.intf1_smac : cfg.intf2_smac) : smac;
        dmac = use_d ? mac48(c2s ? cfg.intf1_dmac : cfg.intf2_dmac) : dmac;
        // subsmac: the list in order, each entry seeing the earlier entries' rewrites
        for (int e = 0; e < cfg.n_subs; ++e) {
            const unsigned long long tg = mac48(cfg.subs[e]), rw = mac48(cfg.subs[e] + 6);
            dmac = dmac == tg ? rw : dmac;
            smac = smac == tg ? rw : smac;
        }
        if (cfg.random_set) {  // MAC_MASK_APPLY (en10mb.h:29-30) on the bytes past the kept ones
            const bool us = unicast48(smac), ud = unicast48(dmac);
            unsigned long long s2 = 0, d2 = 0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {  // per byte, u8 arithmetic (the subtraction wraps in the byte)
                const u32 m = i >= cfg.random_keep ? (u32)cfg.random_mask[i] : 0u;
                const u32 mS = us ? m : 0u, mD = ud ? m : 0u;
                const u32 xs = (u32)(smac >> (8 * i)) & 0xffu, xd = (u32)(dmac >> (8 * i)) & 0xffu;
                s2 |= (unsigned long long)(((xs ^ mS) - (xs & mS)) & 0xffu) << (8 * i);
                d2 |= (unsigned long long)(((xd ^ mD) - (xd & mD)) & 0xffu) << (8 * i);
            }
            smac = s2;
            dmac = d2;
            if (!cfg.random_keep) {
                smac &= us ? ~1ull : ~0ull;
                dmac &= ud ? ~1ull : ~0ull;
            }
        }
        H[0] = with_hi16(H[0], (u32)dmac);
        H[1] = (u32)(dmac >> 16);
        H[2] = (u32)smac;
        H[3] = with_lo16(H[3], (u32)(smac >> 32));
        dirty |= 0xfu;
    }

    // F_INCR (no --fixcsum): the IPv4 header and TCP checksum fields follow the
    // incremental updates too, and a packet is recomputed only when an edit asks for it
    // (needtorecalc: a TTL/hop-limit change, tcpedit.c:195,211)
    constexpr bool kIncr = (F & F_INCR) != 0;
    u32 ics = hi16(H[6]);  // IPv4 header checksum (IP + 10), raw LE
    bool recalc = false;
    // ---- IP header edits (tcpedit.c:184-237), before the port map ----
    if ((F & F_HDR) && cfg.tos > -1) {  // TOS (IPv4) + csum_replace2
        const u32 oldv = lo16(H[4]), newv = (oldv & 0xffu) | ((u32)(cfg.tos & 0xff) << 8);
        H[4] = v6 ? H[4] : with_lo16(H[4], newv);
        if (kIncr) ics = v6 ? ics : (u32)csum_replace2_v((u16)ics, (u16)oldv, (u16)newv);
        dirty |= v6 ? 0u : 1u << 4;
    }
    if ((F & F_HDR) && cfg.ttl_mode != TE_TTL_OFF) {  // rewrite_ipv4_ttl / rewrite_ipv6_hlim (edit_packet.c:627-706)
        const u32 t0 = v6 ? H[5] >> 24 : H[6] & 0xffu, v = cfg.ttl_value & 0xffu;
        u32 t = t0;
        bool changed = true;
        if (cfg.ttl_mode == TE_TTL_SET) {
            changed = t0 != v;
            t = v;
        } else if (cfg.ttl_mode == TE_TTL_ADD) {
            t = t0 + v > 255u ? 255u : t0 + v;
        } else {
            t = t0 <= v ? 1u : t0 - v;
        }
        H[5] = v6 ? ((H[5] & 0x00ffffffu) | (t << 24)) : H[5];
        H[6] = v6 ? H[6] : ((H[6] & ~0xffu) | t);
        if (kIncr) ics = (v6 || !changed) ? ics : (u32)csum_replace2_v((u16)ics, (u16)t0, (u16)t);
        recalc = changed;
        dirty |= v6 ? 1u << 5 : 1u << 6;
    }
    if ((F & F_HDR) && cfg.tclass > -1) {  // tcpedit.c:214-228
        const u32 f = (bswap32(H[4]) & 0xf00fffffu) + ((u32)cfg.tclass << 20);
        H[4] = v6 ? bswap32(f) : H[4];
        dirty |= v6 ? 1u << 4 : 0u;
    }
    if ((F & F_HDR) && cfg.flowlabel > -1) {  // tcpedit.c:231-237
        const u32 f = (bswap32(H[4]) & 0xfff00000u) + (u32)cfg.flowlabel;
        H[4] = v6 ? bswap32(f) : H[4];
        dirty |= v6 ? 1u << 4 : 0u;
    }

    // ---- --mtu-trunc: the IP length fields of the cut packet (a full recompute follows:
    // untrunc_packet's 1 is a needtorecalc) ----
    // (selects, not a branch on the lane's cut: see the note above phase_a)
    H[4] = (cut & !v6) ? with_hi16(H[4], bs16(tcap - 14u)) : H[4];
    H[5] = (cut & v6) ? with_lo16(H[5], bs16(tcap - 54u)) : H[5];
    dirty |= cut ? (v6 ? 1u << 5 : 1u << 4) : 0u;
    // L4 header (20 bytes) at packet offset 34 (v4) or 54 (v6)
    // bitwise selects, not `v6 ? H[14+i] : H[9+i]`: the compiler folds the
    // latter into one dynamically indexed access, which moves H to scratch
    const u32 m6 = v6 ? 0xffffffffu : 0u;
    u32 L[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) L[i] = (H[14 + i] & m6) | (H[9 + i] & ~m6);
    u32 ucs = hi16(L[1]);  // UDP checksum field (L4 + 6), raw LE
    u32 tcs = lo16(L[4]);  // TCP checksum field (L4 + 16), raw LE (F_INCR)
    const bool udp_live = !tcp;

    // ---- port map (rewrite_ports, portmap.c:267-330): destination, then source ----
    if ((F & F_PORTMAP) && cfg.has_portmap) {
        const u32 od = hi16(L[0]), os = lo16(L[0]);
        u32 nd = od, ns = os;
        if (cfg.n_pm >= 0) {
            // the map's few non-identity entries, from LDS (unique keys: at most one hit
            // each).  A LUT load from HBM would wait behind the next tile's loads in flight.
            for (int i = 0; i < cfg.n_pm; ++i) {
                const u32 f = cfg.pm_from[i], to = cfg.pm_to[i];
                nd = f == od ? to : nd;
                ns = f == os ? to : ns;
            }
        } else {
            nd = lut[od];
            ns = lut[os];
            // consume the loads here, so their wait stays on this path (a wait after the
            // merge would also drain the next tile's loads on the LDS path)
            asm volatile("" : "+v"(nd), "+v"(ns));
        }
        ucs = ((nd != od) & udp_live & (ucs != 0)) ? (u32)csum_replace2_v((u16)ucs, (u16)od, (u16)nd) : ucs;
        if (kIncr) tcs = ((nd != od) & tcp) ? (u32)csum_replace2_v((u16)tcs, (u16)od, (u16)nd) : tcs;
        L[0] = with_hi16(L[0], nd);
        ucs = ((ns != os) & udp_live & (ucs != 0)) ? (u32)csum_replace2_v((u16)ucs, (u16)os, (u16)ns) : ucs;
        if (kIncr) tcs = ((ns != os) & tcp) ? (u32)csum_replace2_v((u16)tcs, (u16)os, (u16)ns) : tcs;
        L[0] = with_lo16(L[0], ns);
    }
    if ((F & F_HDR) && cfg.tcp_sequence_enable) {  // rewrite_seqs (rewrite_sequence.c:37-55), TCP only
        const u32 os = L[1], ns = bswap32(bswap32(os) + cfg.tcp_sequence_adjust);
        tcs = tcp ? (u32)csum_replace4_v((u16)tcs, os, ns) : tcs;
        L[1] = tcp ? ns : L[1];
        const u32 fl = (L[3] >> 8) & 0xffu;
        const bool ack = tcp & !((fl & 0x02u) && !(fl & 0x10u));
        const u32 oa = L[2], na = bswap32(bswap32(oa) + cfg.tcp_sequence_adjust);
        tcs = ack ? (u32)csum_replace4_v((u16)tcs, oa, na) : tcs;
        L[2] = ack ? na : L[2];
        dirty |= 0x6u << (v6 ? 14 : 9);
    }

    constexpr bool kAddr = (F & (F_RWIP | F_SEED)) != 0;
    const bool edit_addr = kAddr && (((F & F_RWIP) && cfg.rewrite_ip) || ((F & F_SEED) && kn.seed));
    if (edit_addr && __ballot(!v6)) {
        u32 src = H[7], dst = H[8];
        // ipv4_addr_csum_replace's L4 part (edit_packet.c:259-296): only the UDP field is
        // carried, and only on an IPv4 lane whose address was replaced
#define FL_V4_UPD(c, o, n)                                                                          \
    ucs = ((c) & !v6 & udp_live & (ucs != 0)) ? (u32)csum_replace4_v((u16)ucs, (o), (n)) : ucs;    \
    if (kIncr) {                                                                                    \
        ics = ((c) & !v6) ? (u32)csum_replace4_v((u16)ics, (o), (n)) : ics;                         \
        tcs = ((c) & !v6 & tcp) ? (u32)csum_replace4_v((u16)tcs, (o), (n)) : tcs;                   \
    }
        if ((F & F_RWIP) && cfg.rewrite_ip) {  // rewrite_ipv4l3 (edit_packet.c:787-878)
            bool done = false;  // the first matching entry of each list
            for (int m = 0; m < cfg.n_srcipmap; ++m) {
                const bool hit = !done & ip_in_cidr_f(cfg.srcipmap[m].from, src);
                const u32 o = src, n = remap_ipv4_f(kn, cfg.srcipmap[m].to, o);
                src = hit ? n : o;
                FL_V4_UPD(hit, o, n);
                done |= hit;
            }
            done = false;
            for (int m = 0; m < cfg.n_dstipmap; ++m) {
                const bool hit = !done & ip_in_cidr_f(cfg.dstipmap[m].from, dst);
                const u32 o = dst, n = remap_ipv4_f(kn, cfg.dstipmap[m].to, o);
                dst = hit ? n : o;
                FL_V4_UPD(hit, o, n);
                done |= hit;
            }
            if (cfg.n_cidrmap1 != 0) {
                // the reference walks both lists in step, each index stopping at its list's
                // end, until both addresses matched or both lists ran out: max(n1, n2) steps
                const int n1 = c2s ? cfg.n_cidrmap1 : cfg.n_cidrmap2, n2 = c2s ? cfg.n_cidrmap2 : cfg.n_cidrmap1;
                const int steps = cfg.n_cidrmap1 > cfg.n_cidrmap2 ? cfg.n_cidrmap1 : cfg.n_cidrmap2;
                bool diddst = false, didsrc = false;
                for (int k = 0; k < steps; ++k) {
                    const int i1 = k < n1 - 1 ? k : (n1 > 0 ? n1 - 1 : 0);
                    const int i2 = k < n2 - 1 ? k : (n2 > 0 ? n2 - 1 : 0);
                    const te_cidrmap_t &e2 = c2s ? cfg.cidrmap2[i2] : cfg.cidrmap1[i2];
                    const te_cidrmap_t &e1 = c2s ? cfg.cidrmap1[i1] : cfg.cidrmap2[i1];
                    const bool hd = !diddst & ip_in_cidr_f(e2.from, dst);
                    {
                        const u32 o = dst, n = remap_ipv4_f(kn, e2.to, o);
                        dst = hd ? n : o;
                        FL_V4_UPD(hd, o, n);
                    }
                    diddst |= hd;
                    const bool hs = !didsrc & ip_in_cidr_f(e1.from, src);
                    {
                        const u32 o = src, n = remap_ipv4_f(kn, e1.to, o);
                        src = hs ? n : o;
                        FL_V4_UPD(hs, o, n);
                    }
                    didsrc |= hs;
                }
            }
        }
        if ((F & F_SEED) && kn.seed) {  // randomize_ipv4 (edit_packet.c:420-467): destination, then source
            // a skipped address maps to itself, and the update of an unchanged address
            // leaves the checksum field as it is
            {
                const u32 o = dst;
                dst = (kn.skip_bcast && mcast4(o)) ? o : randomize_ipv4_sw(kn.seed_sw, o);
                FL_V4_UPD(true, o, dst);
            }
            {
                const u32 o = src;
                src = (kn.skip_bcast && mcast4(o)) ? o : randomize_ipv4_sw(kn.seed_sw, o);
                FL_V4_UPD(true, o, src);
            }
        }
#undef FL_V4_UPD
        H[7] = v6 ? H[7] : src;
        H[8] = v6 ? H[8] : dst;
        dirty |= v6 ? 0u : (1u << 7) | (1u << 8);
    }
    if (edit_addr && __ballot(v6)) {
        u32 src[4] = {H[6], H[7], H[8], H[9]}, dst[4] = {H[10], H[11], H[12], H[13]};
        // ipv6_addr_csum_replace (edit_packet.c:298-330): only the UDP field is carried
#define FL_V6_UPD(c, o, n)                                                                          \
    ucs = ((c) & v6 & udp_live & (ucs != 0)) ? (u32)csum_replace16_v((u16)ucs, (o), (n)) : ucs;    \
    if (kIncr) tcs = ((c) & v6 & tcp) ? (u32)csum_replace16_v((u16)tcs, (o), (n)) : tcs
#define FL_V6_SET(a, c, n)                                 \
    _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) a[q_] = (c) ? n[q_] : a[q_];
        if ((F & F_RWIP) && cfg.rewrite_ip) {  // rewrite_ipv6l3 (edit_packet.c:884-1019); TCP/UDP: no ICMPv6 recursion
            bool done = false;
            for (int m = 0; m < cfg.n_srcipmap; ++m) {
                const bool hit = !done & ip6_in_cidr_w(cfg.srcipmap[m].from, src);
                u32 n[4] = {src[0], src[1], src[2], src[3]};
                remap_ipv6_w(kn, cfg.srcipmap[m].to, n);
                FL_V6_UPD(hit, src, n);
                FL_V6_SET(src, hit, n);
                done |= hit;
            }
            done = false;
            for (int m = 0; m < cfg.n_dstipmap; ++m) {
                const bool hit = !done & ip6_in_cidr_w(cfg.dstipmap[m].from, dst);
                u32 n[4] = {dst[0], dst[1], dst[2], dst[3]};
                remap_ipv6_w(kn, cfg.dstipmap[m].to, n);
                FL_V6_UPD(hit, dst, n);
                FL_V6_SET(dst, hit, n);
                done |= hit;
            }
            if (cfg.n_cidrmap1 != 0) {
                const int n1 = c2s ? cfg.n_cidrmap1 : cfg.n_cidrmap2, n2 = c2s ? cfg.n_cidrmap2 : cfg.n_cidrmap1;
                const int steps = cfg.n_cidrmap1 > cfg.n_cidrmap2 ? cfg.n_cidrmap1 : cfg.n_cidrmap2;
                bool diddst = false, didsrc = false;
                for (int k = 0; k < steps; ++k) {
                    const int i1 = k < n1 - 1 ? k : (n1 > 0 ? n1 - 1 : 0);
                    const int i2 = k < n2 - 1 ? k : (n2 > 0 ? n2 - 1 : 0);
                    const te_cidrmap_t &e2 = c2s ? cfg.cidrmap2[i2] : cfg.cidrmap1[i2];
                    const te_cidrmap_t &e1 = c2s ? cfg.cidrmap1[i1] : cfg.cidrmap2[i1];
                    const bool hd = !diddst & ip6_in_cidr_w(e2.from, dst);
                    {
                        u32 n[4] = {dst[0], dst[1], dst[2], dst[3]};
                        remap_ipv6_w(kn, e2.to, n);
                        FL_V6_UPD(hd, dst, n);
                        FL_V6_SET(dst, hd, n);
                    }
                    diddst |= hd;
                    const bool hs = !didsrc & ip6_in_cidr_w(e1.from, src);
                    {
                        u32 n[4] = {src[0], src[1], src[2], src[3]};
                        remap_ipv6_w(kn, e1.to, n);
                        FL_V6_UPD(hs, src, n);
                        FL_V6_SET(src, hs, n);
                    }
                    didsrc |= hs;
                }
            }
        }
        if ((F & F_SEED) && kn.seed) {  // randomize_ipv6 (edit_packet.c:469-518): destination, then source
            {
                const bool skip = kn.skip_bcast && (dst[0] & 0xffu) == 0xffu;
                u32 n[4] = {dst[0], dst[1], dst[2], dst[3]};
                randomize_ipv6_w(kn.seed_sw, n);
                FL_V6_UPD(!skip, dst, n);
                FL_V6_SET(dst, !skip, n);
            }
            {
                const bool skip = kn.skip_bcast && (src[0] & 0xffu) == 0xffu;
                u32 n[4] = {src[0], src[1], src[2], src[3]};
                randomize_ipv6_w(kn.seed_sw, n);
                FL_V6_UPD(!skip, src, n);
                FL_V6_SET(src, !skip, n);
            }
        }
#undef FL_V6_SET
#undef FL_V6_UPD
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            H[6 + i] = v6 ? src[i] : H[6 + i];
            H[10 + i] = v6 ? dst[i] : H[10 + i];
        }
        dirty |= v6 ? 0xffu << 6 : 0u;
    }

    // ---- fix_ipv4/ipv6_checksums (edit_packet.c:55-189) -> do_checksum (checksum.c:34-170) ----
    // caplen == len, not a fragment, lengths consistent: the L4 sum always runs,
    // except on a UDP field that is (still) 0 (checksum.c:115).  F_INCR: only for a
    // packet an edit asked to recompute; the others keep the incremental fields.
    const bool full = !kIncr || recalc || force;
    const bool do_l4 = full && (tcp || ucs != 0);
    L[4] = (do_l4 && tcp) ? with_lo16(L[4], 0) : ((kIncr && !full && tcp) ? with_lo16(L[4], tcs) : L[4]);
    ucs = (do_l4 && !tcp) ? 0u : ucs;                     // uh_sum (L4 + 6)
    L[1] = tcp ? L[1] : with_hi16(L[1], ucs);             // (TCP: the sequence number's low half)
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        H[14 + i] = (L[i] & m6) | (H[14 + i] & ~m6);
        H[9 + i] = (L[i] & ~m6) | (H[9 + i] & m6);
    }
    // ports (port map), UDP csum (L4+6), TCP csum (L4+16)
    dirty |= ((((F & F_PORTMAP) && cfg.has_portmap) ? 1u : 0u) | (tcp ? 0x10u : 0x2u)) << (v6 ? 14 : 9);
    // pseudo header: csum_bytes(ip+12, 8) / csum_bytes(ip6+8, 32) + htons(proto + len)
    u32 sum = wsum_acc(H[8], wsum_acc(H[7], 0u));
    if (__ballot(v6)) {
        u32 s6 = 0;
#pragma unroll
        for (int i = 6; i < 14; ++i) s6 = wsum_acc(H[i], s6);
        sum = v6 ? s6 : sum;
    }
    sum += bs16((tcp ? 6u : 17u) + l4len);
    // L4 bytes [L4S, min(caplen, WEND)) inside the window: the whole dwords
    // (4i + 2 <= caplen) and the partly valid one.  Relative offsets 4i - 2 are
    // even, so each dword's halves are packet-pairing 16-bit words.
    const u32 ecap = cut ? tcap : caplen;  // the bytes the checksums cover
#pragma unroll
    for (int i = 9; i < NW; ++i) {
        const bool whole = ecap >= (u32)(4 * i + 2) && (i >= 14 || !v6);
        sum = wsum_acc(whole ? H[i] : 0u, sum);
    }
    sum = wsum_acc(part, sum);  // < 2^16 * 32 overall
    {  // IPv4 header checksum: do_checksum(ip, 0, ip_len) default case over 20 bytes
        const u32 h6 = with_hi16(H[6], 0);
        const u32 hs = wsum_acc(H[8], wsum_acc(H[7], wsum_acc(h6, wsum_acc(H[5], wsum_acc(H[4], 0u)))));
        H[6] = v6 ? H[6] : with_hi16(h6, full ? (~fold32(hs)) & 0xffffu : ics);
        dirty |= v6 ? 0u : 1u << 6;
    }

    // ---- dlt_en10mb_merge_layer3 (en10mb.c:847-887): multicast destination MAC ----
    {
        const u32 d = H[8];
        const bool mc4 = !v6 && mcast4(d), mc6 = v6 && (H[10] & 0xffu) == 0xffu;
        const u32 h1_4 = 0x5eu | (((d >> 8) & 0x7fu) << 8) | (((d >> 16) & 0xffu) << 16) | ((d >> 24) << 24);
        H[0] = mc4 ? with_hi16(H[0], 0x0001u) : (mc6 ? with_hi16(H[0], 0x3333u) : H[0]);  // 01:00 / 33:33
        H[1] = mc4 ? h1_4 : (mc6 ? H[13] : H[1]);
        dirty |= (mc4 || mc6) ? 3u : 0u;
    }

    st.l4sum = sum;
    st.end = ecap;
    st.dirty = dirty;
    st.v6 = v6;
    st.tcp = tcp;
    st.do_l4 = do_l4;
    st.tail = do_l4 && ecap > (u32)WEND;
    return ok;
}

// Phase B: add the L4 bytes past the window (one's-complement sum `tail`,
// already in the packet's relative byte pairing) and store the checksum.
DI void phase_b(u32 (&H)[NW], const State &st, u32 tail) {
    if (!st.do_l4) return;
    const u32 c = (~fold32(st.l4sum + tail)) & 0xffffu;  // CHECKSUM_CARRY (l4sum < 2^22, tail < 2^16)
    // explicit per-index selects (a ternary on the index would move H to scratch)
    const bool t6 = st.tcp && st.v6, t4 = st.tcp && !st.v6, u6 = !st.tcp && st.v6, u4 = !st.tcp && !st.v6;
    H[18] = t6 ? with_lo16(H[18], c) : H[18];  // 54 + 16
    H[13] = t4 ? with_lo16(H[13], c) : H[13];  // 34 + 16
    H[15] = u6 ? with_hi16(H[15], c) : H[15];  // 54 + 6
    H[10] = u4 ? with_hi16(H[10], c) : H[10];  // 34 + 6
}

}  // namespace fl
}  // namespace te
