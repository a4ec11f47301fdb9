// tcpprep_kernels.hip -- gfx950 kernel for tcpprep's per-packet classification
// pass (src/tcpprep.c:339-587 process_raw_packets, per-packet modes).
//
// One lane per cache entry (one pcap record).  A lane locates the record's
// IPv4/IPv6 header with the same L2 chain walk the edit kernels use
// (edit_pkt.hpp: get_l2len_protocol, l4_v4, l4_v6, l4proto_v6, ip_in_cidr),
// applies the include/exclude filter and the mode's test, and yields the 2-bit
// cache entry add_cache (src/common/cache.c:259-314) would store: bit 1 = send,
// bit 0 = C2S.  Four neighbouring lanes OR their entries into one byte with two
// cross-lane shuffles, and the first of them stores it: the output is the
// packed cache body that write_cache (cache.c:146-219) writes after the header.
//
// Bytes per record: the 12-byte index entry, the L2..L4 header bytes the tests
// touch (<= 64 for untagged frames) and a quarter byte of output.  The pass is
// a gather over the capture at record stride, so it is bound by HBM latency
// and the record count, not by the capture's size.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "edit_pkt.hpp"
#include "tp_dev_cfg.h"

namespace {
using namespace te;

DI bool in4(const te_cidr_t *c, int n, u32 ip) {  // check_ip_cidr cidr.c:535-564
    if (n == 0) return true;
    for (int i = 0; i < n; ++i)
        if (ip_in_cidr(c[i], ip)) return true;
    return false;
}

DI bool in6(const te_cidr_t *c, int n, const u8 *a) {  // check_ip6_cidr cidr.c:570-598
    if (n == 0) return true;
    for (int i = 0; i < n; ++i)
        if (ip6_in_cidr(c[i], a)) return true;
    return false;
}

DI bool check_list(const tp_dev_cfg_t &c, uint64_t v) {  // list.c:139-156
    for (int i = 0; i < c.nlist; ++i) {
        uint64_t mn = c.lmin[i], mx = c.lmax[i];
        if (mn != 0 && mx != 0) {
            if (v >= mn && v <= mx) return true;
        } else if (mn == 0) {
            if (v <= mx) return true;
        } else if (v >= mn) {
            return true;
        }
    }
    return false;
}

// process_xX_by_cidr_ipv4/ipv6 (xX.c:124-236): true = SEND
DI bool xx_cidr(const tp_dev_cfg_t &c, const u8 *ip, bool v6) {
    bool s, d;
    if (v6) {
        s = in6(c.xx_cidr, c.nxx_cidr, ip + 8);
        d = in6(c.xx_cidr, c.nxx_cidr, ip + 24);
    } else {
        s = in4(c.xx_cidr, c.nxx_cidr, ld32(ip + 12));
        d = in4(c.xx_cidr, c.nxx_cidr, ld32(ip + 16));
    }
    const bool ex = (c.xx_mode & TP_XX_EXCLUDE) != 0;
    bool hit;
    switch (c.xx_mode & ~TP_XX_EXCLUDE) {
        case TP_XX_SOURCE: hit = s; break;
        case TP_XX_DEST: hit = d; break;
        case TP_XX_BOTH: hit = d && s; break;
        case TP_XX_EITHER: hit = d || s; break;
        default: return !ex;  // "Unable to determine action in CIDR filter mode"
    }
    return ex ? !hit : hit;
}

DI bool svc(const uint32_t *bits, u32 port) { return (bits[port >> 5] >> (port & 31)) & 1u; }

// check_dst_port (tcpprep.c:211-295): 1 = C2S, 0 = S2C, or --nonip's value
DI int dst_port(const tp_dev_cfg_t &c, const u8 *ip, bool v6, int len) {
    int l4;
    u8 proto;
    if (!v6) {
        if (len < ((ip[0] & 0x0f) * 4) + 4) return 0;
        proto = ip[9];
        l4 = l4_v4(ip, len);
    } else {
        if (len < 40 + 4) return 0;
        proto = l4proto_v6(ip, len);
        l4 = l4_v6(ip, 0, len);
    }
    if (l4 < 0) return 0;
    if (proto == 6) {
        if (len - l4 < 20) return 0;
        return svc(c.svc_tcp, be16(ip + l4 + 2)) ? 1 : 0;
    }
    if (proto == 17) {
        if (len - l4 < 8) return 0;
        return svc(c.svc_udp, be16(ip + l4 + 2)) ? 1 : 0;
    }
    return c.nonip;
}


// ---------------------------------------------------------------------------
// Auto modes (tree.c).  First pass: every IP record inserts its source (and in
// first mode its destination) into an open-addressing table on exact 64-bit
// keys and bumps the node's counters; the table is the RB tree's set of
// nodes, and atomics make the order of insertion irrelevant except where the
// reference is order-dependent (first mode), which an atomicMax over the complement of the
// sighting order reproduces.  A node's key and counts share one 16-byte pair, so the
// counter update hits the line its insertion just brought into L2.  Second pass (classify): tree_calculate + check_ip_tree
// per record from its source's slot.
// ---------------------------------------------------------------------------
constexpr uint64_t TP_V6_KEY = 1ull << 62;

DI uint64_t node_key(bool v6, const u8 *addr) { return v6 ? TP_V6_KEY : (1ull << 63) | (uint64_t)ld32(addr); }

DI uint32_t tree_insert(const tp_tree_t &t, uint64_t key) {
    uint64_t h = key * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    for (uint64_t k = 0; k <= t.mask; ++k) {
        const uint64_t s = (h + k) & t.mask;
        const uint64_t prev = atomicCAS((unsigned long long *)&t.slots[2 * s], 0ull, (unsigned long long)key);
        if (prev == 0 || prev == key) return (uint32_t)s;
    }
    return 0xffffffffu;  // cannot happen: capacity >= 2x the insertions
}

// get_l2len_protocol over the capture's link type (get.c:263-452): the L3 protocol and
// the bytes before the IP header, for every DLT tcpprep reads (tcpprep.c:108-118).  A
// Juniper record without an L2 header never gets here (the host refuses the capture: the
// reference's get_ipv4 then reads ~4 GiB past the packet, get.c:509-510)
DI int tp_l2(const u8 *d, u32 caplen, int dlt, L2 &r) {
    r.protocol = 0;
    r.l2len = 0;
    if (!caplen) return -1;
    switch (dlt) {
    case 1:  // DLT_EN10MB
        return get_l2len_protocol(d, caplen, r);
    case 12:   // DLT_RAW (linktype 101)
    case 101:
        r.protocol = (d[0] >> 4) == 4 ? 0x0800 : (d[0] >> 4) == 6 ? 0x86DD : 0;
        return 0;
    case 50:  // DLT_PPP_SERIAL: the PPP IPv4 protocol number counts as IPv4
        if (caplen < 4) return -1;
        r.l2len = 4;
        r.protocol = be16(d + 2) == 0x0021 ? 0x0800 : be16(d + 2);
        return 0;
    case 104:  // DLT_C_HDLC
        if (caplen < 4) return -1;
        r.l2len = 4;
        r.protocol = be16(d + 2);
        return 0;
    case 113:  // DLT_LINUX_SLL
        if (caplen < 16) return -1;
        r.l2len = 16;
        r.protocol = be16(d + 14);
        return 0;
    case 276:  // DLT_LINUX_SLL2
        if (caplen < 20) return -1;
        r.l2len = 20;
        r.protocol = be16(d);
        return 0;
    case 178: {  // DLT_JUNIPER_ETHER: magic, flags, extensions, then the Ethernet header
        if (caplen < 4 || d[0] != 0x4d || d[1] != 0x47 || d[2] != 0x43) return -1;
        u32 off = 4;
        if (d[3] & 0x80) {
            if (caplen < 6) return -1;
            off = (u32)be16(d + 4) + 6;
        }
        if (d[3] & 0x02) return -1;
        if (caplen <= off + 18) return -1;  // datalen <= l2_net_off + 4
        if (get_l2len_protocol(d + off, caplen - off, r) == -1) return -1;
        r.l2len += off;
        return 0;
    }
    default:
        return -1;
    }
}

// packet2tree (tree.c:653-838): node type for the source, -1 unknown, -2 len_error
DI int packet2tree(const u8 *d, u32 caplen, int dlt) {
    L2 r;
    if (tp_l2(d, caplen, dlt, r) == -1) return -2;
    const long len = caplen;
    long hl = 0;
    u8 proto = 0;
    if (r.protocol == 0x0800) {
        if (len < (long)r.l2len + 20) return -2;
        proto = d[r.l2len + 9];
        hl = (d[r.l2len] & 0x0f) * 4;
    } else if (r.protocol == 0x86DD) {
        if (len < (long)r.l2len + 40) return -2;
        proto = d[r.l2len + 6];
        hl = 40;
    }
    const long l4 = (long)r.l2len + hl;
    if (proto == 6) {
        if (len < l4 + 20) return -2;
        if (ld16(d + l4) == 20) return -1;  // th_sport == 20 without ntohs (ftp-data)
        const u8 fl = d[l4 + 13];
        return fl == 0x02 ? 0 : fl == 0x12 ? 1 : -1;
    }
    if (proto == 17) {
        if (len < l4 + 8) return -2;
        if (be16(d + l4 + 2) == 53) {
            if (len < l4 + 8 + 12) return -2;
            return (ld16(d + l4 + 10) & 0x8000) ? 1 : 0;  // dnsv4_hdr.flags unswapped
        }
        if (be16(d + l4) == 53) {
            if (len < l4 + 8 + 12) return -2;
            return ((ld16(d + l4 + 10) & 0x7FFFF) ^ 0x8000) ? 1 : 0;
        }
        return -1;
    }
    if (proto == 1) {
        if (len < l4 + 4) return -2;
        if (d[l4] == 3 && d[l4 + 1] == 3) return 1;  // port unreachable
    }
    return -1;
}

__global__ __launch_bounds__(256) void tp_tree_build(const u8 *__restrict__ img, const uint64_t *__restrict__ off,
                                                     const uint32_t *__restrict__ caplen, uint64_t n, int first_mode,
                                                     uint64_t base, tp_tree_t t, const tp_dev_cfg_t *cfg) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const tp_dev_cfg_t &c = *cfg;
    // the include/exclude filters skip a record before the tree (tcpprep.c:362-375, 413-428;
    // that first pass's DONT_SEND entries are the host's, tcpprep_cache_pcap)
    if (c.nlist && check_list(c, c.pkt_base + j + 1) == ((c.xx_mode & TP_XX_EXCLUDE) != 0)) {
        t.slot[j] = 0xffffffffu;
        return;
    }
    const u8 *d = img + off[j];
    const u32 cl = caplen[j];
    const int dlt = c.dlt;
    L2 r;
    const int res = cl ? tp_l2(d, cl, dlt, r) : -1;
    const bool v4 = res != -1 && r.l2len + 20 <= cl && r.protocol == 0x0800;
    const bool v6 = !v4 && res != -1 && r.l2len + 40 <= cl && r.protocol == 0x86DD;
    if (!v4 && !v6) {
        t.slot[j] = 0xffffffffu;
        return;
    }
    const u8 *ip = d + r.l2len;
    if (c.nxx_cidr && c.xx_mode && !xx_cidr(c, ip, v6)) {
        t.slot[j] = 0xffffffffu;
        return;
    }
    const uint32_t s = tree_insert(t, node_key(v6, ip + (v6 ? 8 : 12)));
    t.slot[j] = s;
    if (s == 0xffffffffu) {
        atomicMin((unsigned long long *)t.err, (unsigned long long)j);
        return;
    }
    if (first_mode) {  // add_tree_first_ipv4/ipv6 (tree.c:333-452): the first sighting decides
        // (base: the shard's global record index, so shards' sightings merge by order)
        atomicMax((unsigned long long *)&t.slots[2 * s + 1], ~(unsigned long long)(2 * (base + j)));  // ~min = max ~
        const uint32_t sd = tree_insert(t, node_key(v6, ip + (v6 ? 24 : 16)));
        if (sd == 0xffffffffu)
            atomicMin((unsigned long long *)t.err, (unsigned long long)j);
        else
            atomicMax((unsigned long long *)&t.slots[2 * sd + 1], ~(unsigned long long)(2 * (base + j) + 1));
        return;
    }
    const int ty = packet2tree(d, cl, dlt);  // add_tree_ipv4/ipv6 + add_tree_node (tree.c:454-538)
    if (ty == -2)
        atomicMin((unsigned long long *)t.err, (unsigned long long)j);
    else if (ty >= 0)  // the counts share the key's 16-byte pair: one line per node
        atomicAdd((unsigned long long *)&t.slots[2 * s + 1], ty == 1 ? 1ull << 32 : 1ull);
}

// sharded auto modes: a node's value from the table merged across ranks (binary search)
__global__ __launch_bounds__(256) void tp_tree_merged(tp_tree_t t, uint64_t cap, const uint64_t *__restrict__ keys,
                                                      const uint64_t *__restrict__ vals, uint64_t n) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    const uint64_t key = t.slots[2 * s];
    if (!key) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (keys[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    if (lo < n && keys[lo] == key) t.slots[2 * s + 1] = vals[lo];
}

// tree_calculate (tree.c:540-565) + check_ip_tree (:219-272): the tcpr_dir_t of a source
DI int tree_dir(const tp_dev_cfg_t &c, const tp_tree_t &t, uint32_t s) {
    uint32_t sc, cc;
    const uint64_t w = t.slots[2 * s + 1];
    if (c.automode == TP_AUTO_FIRST) {
        const bool dst_first = ~w & 1;
        sc = dst_first ? 1000 : 0;
        cc = dst_first ? 0 : 1000;
    } else {
        sc = (uint32_t)(w >> 32);
        cc = (uint32_t)w;
    }
    if (sc > 0 || cc > 0) return (double)sc >= (double)cc * c.ratio ? 2 : 1;  // server: S2C, client: C2S
    // router: process_tree (tree.c:156-203) builds CIDRs whose family new_cidr() leaves 0, so
    // nothing is ever "in" them and it succeeds at --maxmask; the second pass is then
    // check_ip_tree(options->nonip, ...) (tcpprep.c:498-509): DIR_CLIENT, or DIR_SERVER with --nonip
    if (c.automode == TP_AUTO_ROUTER) return c.nonip ? 2 : 1;
    return c.automode == TP_AUTO_SERVER ? 2 : c.automode == TP_AUTO_CLIENT ? 1 : -1;
}

// ---- --regex (tcpprep.c:300-335): the source address as inet_ntop prints it, through
// the host-compiled DFA (tp_regex.c) one character at a time ----
DI int dstep(const u8 *T, int st, int k) { return T[st * TP_NSYM + k]; }
DI int ddec(const u8 *T, int st, u32 v) {  // "%u" of an octet
    if (v >= 100) st = dstep(T, st, (int)(v / 100));
    if (v >= 10) st = dstep(T, st, (int)((v / 10) % 10));
    return dstep(T, st, (int)(v % 10));
}
DI int dhex(const u8 *T, int st, u32 w) {  // "%x" of a 16-bit word
    bool lead = true;
    for (int sh = 12; sh >= 0; sh -= 4) {
        const u32 d = (w >> sh) & 15u;
        if (d || !lead || sh == 0) {
            st = dstep(T, st, (int)d);
            lead = false;
        }
    }
    return st;
}
DI int dv4(const u8 *T, int st, const u8 *a) {  // inet_ntop4: dotted decimal
    for (int i = 0; i < 4; ++i) {
        if (i) st = dstep(T, st, 16);
        st = ddec(T, st, a[i]);
    }
    return st;
}
// glibc inet_ntop6: the first longest run (>= 2) of zero words becomes "::"; an
// IPv4-compatible (::a.b.c.d) or -mapped (::ffff:a.b.c.d) address ends in dotted form
DI bool regex_match(const u8 *T, int start, const u8 *ip, bool v6) {
    int st = dstep(T, start, TP_SYM_BOS);
    if (!v6) {
        st = dv4(T, st, ip + 12);
    } else {
        const u8 *a = ip + 8;
        u32 w[8];
        for (int i = 0; i < 8; ++i) w[i] = ((u32)a[2 * i] << 8) | a[2 * i + 1];
        int bb = -1, bl = 0, cb = -1, cl = 0;
        for (int i = 0; i < 8; ++i) {
            if (w[i] == 0) {
                if (cb < 0) cb = i, cl = 1;
                else ++cl;
            } else if (cb >= 0) {
                if (bb < 0 || cl > bl) bb = cb, bl = cl;
                cb = -1;
            }
        }
        if (cb >= 0 && (bb < 0 || cl > bl)) bb = cb, bl = cl;
        if (bb >= 0 && bl < 2) bb = -1;
        for (int i = 0; i < 8; ++i) {
            if (bb >= 0 && i >= bb && i < bb + bl) {
                if (i == bb) st = dstep(T, st, 17);
                continue;
            }
            if (i) st = dstep(T, st, 17);
            if (i == 6 && bb == 0 && (bl == 6 || (bl == 5 && w[5] == 0xffffu))) {
                st = dv4(T, st, a + 12);
                break;
            }
            st = dhex(T, st, w[i]);
        }
        if (bb >= 0 && bb + bl == 8) st = dstep(T, st, 17);
    }
    return dstep(T, st, TP_SYM_EOS) == 0;
}

// one record -> its 2-bit cache entry
DI u32 classify(const tp_dev_cfg_t &c, const tp_tree_t *t, uint64_t j, const u8 *pkt, u32 caplen,
                 uint64_t pktnum, const u8 *dfa) {
    constexpr u32 SEND = 2, C2S = 1;
    // include/exclude packet list (tcpprep.c:362-375)
    if (c.nlist && check_list(c, pktnum) == ((c.xx_mode & TP_XX_EXCLUDE) != 0)) return 0;
    int dir;
    if (c.mode != TP_MODE_MAC) {
        L2 r;
        const int res = caplen ? tp_l2(pkt, caplen, c.dlt, r) : -1;
        const bool v4 = res != -1 && r.l2len + 20 <= caplen && r.protocol == 0x0800;  // get_ipv4 get.c:483-541
        const bool v6 = !v4 && res != -1 && r.l2len + 40 <= caplen && r.protocol == 0x86DD;  // get_ipv6 :550-608
        if (!v4 && !v6) return SEND | (c.nonip == 1 ? C2S : 0);  // add_cache(SEND, options->nonip)
        const u8 *ip = pkt + r.l2len;
        if (c.nxx_cidr && c.xx_mode && !xx_cidr(c, ip, v6)) return 0;
        if (c.mode == TP_MODE_AUTO) {
            dir = tree_dir(c, *t, t->slot[j]);  // -1 (TCPR_DIR_ERROR): send bit only
        } else if (c.mode == TP_MODE_REGEX) {
            // check_ipv4_regex / check_ipv6_regex return 1 or 0; --reverse swaps only 1 and 2
            // (tcpprep.c:441-442), so a reversed match (2) and a miss (0) both leave the
            // direction bit clear (add_cache, cache.c:292)
            dir = regex_match(dfa, c.dfa.start, ip, v6) ? 1 : 0;
            if (c.reverse && dir == 1) dir = 2;
        } else if (c.mode == TP_MODE_CIDR) {
            dir = v6 ? in6(c.cidr, c.ncidr, ip + 8) : in4(c.cidr, c.ncidr, ld32(ip + 12));
            if (c.reverse) dir = !dir;
        } else {
            dir = dst_port(c, ip, v6, (int)caplen - (int)r.l2len);
        }
    } else {  // macinstring (mac.c:76-115) on the source MAC; caplen < 14 records are not indexed
        dir = 0;
        if (!c.mac_first_empty)
            for (int m = 0; m < c.nmac; ++m) {
                const u8 *a = c.mac[m];
                bool eq = true;
                for (int b = 0; b < 6; ++b) eq &= pkt[6 + b] == a[b];
                if (eq) {
                    dir = 1;
                    break;
                }
            }
        if (c.reverse) dir = !dir;
    }
    return SEND | (dir == 1 ? C2S : 0);
}

__global__ __launch_bounds__(256) void tp_classify(const u8 *__restrict__ img, const uint64_t *__restrict__ off,
                                                   const uint32_t *__restrict__ caplen,
                                                   const uint32_t *__restrict__ pktnum, uint64_t n,
                                                   const tp_dev_cfg_t *__restrict__ cfg, const tp_tree_t *tree,
                                                   u8 *__restrict__ out) {
    // the --regex DFA in LDS (5 KiB): one dependent lookup per address character
    __shared__ __attribute__((aligned(16))) u8 dfa[TP_DFA_MAX * TP_NSYM];
    if (cfg->mode == TP_MODE_REGEX) {
        const u32 *src = (const u32 *)&cfg->dfa.next[0][0];
        for (u32 i = threadIdx.x; i < sizeof(dfa) / 4; i += blockDim.x) ((u32 *)dfa)[i] = src[i];
        __syncthreads();
    }
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    u32 e = 0;
    if (j < n)
        e = classify(*cfg, tree, j, img + off[j], caplen[j], cfg->pkt_base + (pktnum ? (uint64_t)pktnum[j] : j + 1),
                     dfa);
    e <<= 2 * (j & 3);
    e |= __shfl_xor(e, 1);
    e |= __shfl_xor(e, 2);
    if ((j & 3) == 0 && j < n) out[j >> 2] = (u8)e;
}
}  // namespace

extern "C" int tp_launch_classify(const uint8_t *img, const uint64_t *off, const uint32_t *caplen,
                                  const uint32_t *pktnum, uint64_t n_entries, const tp_dev_cfg_t *cfg,
                                  const tp_tree_t *tree, uint8_t *out, void *stream) {
    if (n_entries == 0) return 0;
    const uint64_t blocks = (n_entries + 255) / 256;
    if (blocks > 0x7fffffffull) return -1;
    hipLaunchKernelGGL(tp_classify, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, img, off, caplen, pktnum,
                       n_entries, cfg, tree, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int tp_launch_tree_merged(tp_tree_t tree, uint64_t capacity, const uint64_t *keys, const uint64_t *vals,
                                     uint64_t n, void *stream) {
    if (capacity == 0) return 0;
    hipLaunchKernelGGL(tp_tree_merged, dim3((unsigned)((capacity + 255) / 256)), dim3(256), 0, (hipStream_t)stream, tree,
                       capacity, keys, vals, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int tp_launch_tree(const uint8_t *img, const uint64_t *off, const uint32_t *caplen, uint64_t n_entries,
                              const tp_dev_cfg_t *cfg, int automode, uint64_t base, tp_tree_t tree, void *stream) {
    if (n_entries == 0) return 0;
    const uint64_t blocks = (n_entries + 255) / 256;
    if (blocks > 0x7fffffffull) return -1;
    hipLaunchKernelGGL(tp_tree_build, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, img, off, caplen,
                       n_entries, automode == TP_AUTO_FIRST ? 1 : 0, base, tree, cfg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
