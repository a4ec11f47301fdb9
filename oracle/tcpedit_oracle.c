/*
 * tcpedit_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never shipped).
 *
 * A plain-C, single-threaded CPU restatement of the reference's per-packet
 * edit path: libtcpedit's tcpedit_packet() (src/tcpedit/tcpedit.c:46-366) as
 * driven by tcprewrite's rewrite_packets() (src/tcprewrite.c:260-373), for
 * DLT_EN10MB, LINUX_SLL, LINUX_SLL2, RAW, NULL, LOOP, PPP_SERIAL and C_HDLC input
 * (the decoders of src/tcpedit/plugins/dlt_*) and the en10mb, user, hdlc, pppserial and
 * non-encoding plugins as encoders, --fuzz-seed included
 * (src/tcpedit/fuzzing.c, with the reference's second L2/L3 pass after a fuzz).  Every function cites the reference file:line
 * it restates (paths relative to appneta/tcpreplay 4.5.5).
 *
 * Pinning: this restatement is checked byte-for-byte against the reference's
 * own little-endian golden outputs (test/test2.rewrite_*, committed under
 * tests/golden/) by tests/test_oracle_golden.py.  The reference itself is NOT
 * built here: its path needs libpcap/autogen-generated headers this image lacks,
 * so it is unbuildable without stand-ins (see DESIGN.md "Oracle").
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code.  The product (tcpreplay_amd/, libtcpedit_hip.so) never links
 * or calls it.
 *
 * Like the reference, packets are edited in ONE static MAXPACKET buffer that is
 * reused across packets (src/tcprewrite.c:267-301), so reads past caplen see
 * bytes of earlier packets exactly as the reference does.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

/* ------------------------------------------------------------------------- */
/* constants (src/tcpr.h, src/defines.h.in, src/common/cache.h)              */
/* ------------------------------------------------------------------------- */
#define MAX_SNAPLEN 262144                 /* defines.h.in:177 */
#define MAXPACKET (MAX_SNAPLEN + 22)       /* defines.h.in:182 */
#define DEFAULT_MTU 1500                   /* defines.h.in:171 */
#define DLT_EN10MB 1

#define TCPEDIT_SOFT_ERROR -2              /* tcpedit_types.h:31-34 */
#define TCPEDIT_ERROR -1
#define TCPEDIT_OK 0
#define TCPEDIT_WARN 1

#define DIR_NOSEND 0                       /* cache.h:77-80 */
#define DIR_C2S 1
#define DIR_S2C 2

#define ETHERTYPE_IP 0x0800                /* tcpr.h:510-543 */
#define ETHERTYPE_ARP 0x0806
#define ETHERTYPE_VLAN 0x8100
#define ETHERTYPE_MPLS 0x8847
#define ETHERTYPE_IP6 0x86DD
#define ETHERTYPE_Q_IN_Q 0x88A8
#define ETHERTYPE_8021QINQ 0x9100
#define ETHERTYPE_MPLS_MULTI 0x8848

#define IPPROTO_IP_ 0
#define IPPROTO_ICMP_ 1
#define IPPROTO_TCP_ 6
#define IPPROTO_UDP_ 17
#define IPPROTO_ICMP6_ 58
#define IPPROTO_TCP_V6FRAG 0x2c            /* tcpr.h:655-656 */

#define NH_HBH 0                           /* tcpr.h:777-826 */
#define NH_IPV6 41
#define NH_ROUTING 43
#define NH_FRAGMENT 44
#define NH_ESP 50
#define NH_AH 51
#define NH_NO_NEXT 59
#define NH_DESTOPTS 60

#define IP_MF 0x2000                       /* tcpr.h:706-710 */
#define IP_OFFMASK 0x1fff
#define TH_SYN 0x02
#define TH_ACK 0x10
#define MPLS_LABEL_GACH 13                 /* tcpr.h:1675 */
#define MPLS_LS_S_MASK 0x00000100
#define MPLS_LS_LABEL_SHIFT 12
#define VIDMASK 0x0fff                     /* tcpr.h:147-149 */
#define PRIMASK 0xe000
#define CFIMASK 0x1000

#define TTL_OFF 0                          /* tcpedit_types.h:38-45 */
#define TTL_SET 1
#define TTL_ADD 2
#define TTL_SUB 3
#define FIXLEN_OFF 0
#define FIXLEN_PAD 1
#define FIXLEN_TRUNC 2
#define FIXLEN_DEL 3

#define VLAN_OFF 0                         /* en10mb_types.h:50-54 */
#define VLAN_DEL 1
#define VLAN_ADD 2
#define MASK_SMAC1 1                       /* en10mb_types.h:43-48 */
#define MASK_SMAC2 2
#define MASK_DMAC1 4
#define MASK_DMAC2 8

/* ------------------------------------------------------------------------- */
/* small helpers: unaligned host-order (little-endian) loads/stores          */
/* ------------------------------------------------------------------------- */
static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline void st16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }
static inline void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

/* ------------------------------------------------------------------------- */
/* configuration (restates tcpedit_t tcpedit_types.h:91-153 and             */
/* en10mb_config_t en10mb_types.h:60-92)                                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    int family;       /* 4 or 6 */
    int masklen;
    uint32_t network; /* network byte order, as stored by inet_aton */
    uint8_t network6[16];
} ocidr_t;

typedef struct {
    ocidr_t from, to;
} ocidrmap_t;

typedef struct {
    long from, to; /* network-order values (portmap.c:94-98) */
} oport_t;

typedef struct {
    /* tcpedit_t */
    bool skip_broadcast, rewrite_ip, fixcsum, efcs, mtu_truncate, fixhdrlen;
    int fixlen;
    uint32_t tcp_sequence_enable, tcp_sequence_adjust;
    int ttl_mode;
    uint8_t ttl_value;
    int tos, flowlabel, tclass;
    ocidrmap_t *cidrmap1, *cidrmap2, *srcipmap, *dstipmap;
    int n_cidrmap1, n_cidrmap2, n_srcipmap, n_dstipmap;
    uint32_t seed;
    oport_t *portmap;
    int n_portmap;
    int mtu;
    uint32_t fuzz_seed;     /* tcpedit->fuzz_seed (mixed like the seed, parse_args.c:213-235) */
    uint32_t fuzz_factor;   /* --fuzz-factor, default 8 (tcpedit_opts.def:325-330) */
    /* en10mb_config_t */
    uint8_t intf1_dmac[6], intf1_smac[6], intf2_dmac[6], intf2_smac[6];
    uint8_t (*subs)[2][6];
    int n_subs;
    uint32_t random_set;
    int random_keep;
    uint8_t random_mask[6];
    int mac_mask;
    int vlan;
    uint16_t vlan_tag;
    uint8_t vlan_pri, vlan_cfi;
    uint16_t vlan_proto;
    bool l2_skip_broadcast; /* tcpeditdlt_t.skip_broadcast (--skipl2broadcast) */
    bool skip_soft_errors;
    /* the encoder (tcpedit_dlt_post_args, dlt_plugins.c:168-204): en10mb, user or hdlc */
    int encoder;            /* ENC_EN10MB / ENC_USER / ENC_HDLC */
    int out_linktype;       /* tcpedit_dlt_output_dlt (dlt_plugins.c:268-283) */
    int user_length;        /* user_config_t.length (user_types.h:49-55), -1 = no --user-dlink */
    uint8_t user_l2client[255], user_l2server[255];
    uint16_t hdlc_address, hdlc_control; /* hdlc_config_t (hdlc_types.h), 65535 = unset */
    int user_dlt_set, user_dlt;
    int decoder;            /* DEC_*: the input DLT's plugin (tcpedit_dlt_init, dlt_plugins.c:115-160) */
    int in_dlt;             /* the input DLT (pcap_datalink) */
} ocfg_t;
/* encoders: en10mb, user, hdlc; NOENC = linuxsll/linuxsll2/raw/null/loop, whose encode
   always fails (linuxsll.c:201-208, linuxsll2.c:213-221, raw.c:194-201, null.c:192-198);
   PPP = pppserial, whose encode leaves the packet as it is (pppserial.c:239-251) */
enum { ENC_EN10MB = 0, ENC_USER, ENC_HDLC, ENC_NOENC, ENC_PPP };
/* decoders (NULL and LOOP share dlt_null's functions, loop.c:47-64) */
enum { DEC_EN10MB = 0, DEC_SLL, DEC_SLL2, DEC_RAW, DEC_NULL, DEC_PPP, DEC_CHDLC, DEC_JNPR, DEC_80211, DEC_RADIOTAP };

/* decoder/encoder per-context scratch (tcpeditdlt_t + en10mb_extra_t) which
 * the reference keeps across packets (plugins_types.h:100-131). */
typedef struct {
    uint8_t dstaddr[6], srcaddr[6];
    int proto;          /* ctx->proto */
    int proto_vlan_tag; /* ctx->proto_vlan_tag */
    int l2offset, l2len;
    /* en10mb_extra_t */
    int vlan;
    uint32_t vlan_offset;
    uint16_t vlan_tag, vlan_pri, vlan_cfi, vlan_proto;
    bool src_modified, dst_modified;
    /* DLT_JUNIPER_ETHER: a whole inner decode has been copied in (the encoder's extra is
       the en10mb sub-decoder's from then on, dlt_utils.c:261-263) */
    bool jnpr_sub;
} ostate_t;

typedef struct {
    uint32_t caplen, len;
} ohdr_t;

static __thread char g_err[1024]; /* per thread: a checker runs shards on threads */
static __thread int g_warn_count;

static void seterr(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

/* ------------------------------------------------------------------------- */
/* tcpr_random: src/common/utils.c:436-458                                   */
/* ------------------------------------------------------------------------- */
static uint32_t tcpr_random(uint32_t *seed)
{
    unsigned int next = *seed;
    unsigned int result;
    next *= 1103515245;
    next += 12345;
    result = (int)(next / 65536) % 2048;
    next *= 1103515245;
    next += 12345;
    result <<= 10;
    result ^= (int)(next / 65536) % 1024;
    next *= 1103515245;
    next += 12345;
    result <<= 10;
    result ^= (int)(next / 65536) % 1024;
    *seed = next;
    return result;
}

/* ------------------------------------------------------------------------- */
/* L2 parsing: src/common/get.c:87-451                                       */
/* ------------------------------------------------------------------------- */
/* parse_mpls: get.c:87-157 */
static int parse_mpls(const uint8_t *pkt, uint32_t datalen, uint16_t *next_protocol, uint32_t *l2len, uint32_t *l2offset)
{
    int len = (int)*l2len;
    bool bos = false;
    const uint8_t *label_ptr = NULL;
    while (!bos) {
        if ((uint64_t)len + 4 > datalen)
            return -1;
        label_ptr = pkt + len;
        len += 4;
        uint32_t entry = ntohl(ld32(label_ptr));
        bos = (entry & MPLS_LS_S_MASK) != 0;
        if ((entry >> MPLS_LS_LABEL_SHIFT) == MPLS_LABEL_GACH)
            return -1;
    }
    if ((size_t)(label_ptr + 4 - pkt) + 1 > datalen)
        return -1;
    uint8_t first_nibble = label_ptr[4] >> 4;
    switch (first_nibble) {
    case 4: *next_protocol = ETHERTYPE_IP; break;
    case 6: *next_protocol = ETHERTYPE_IP6; break;
    case 0:
        if ((uint64_t)len + 4 + 14 > datalen)
            return -1;
        len += 4;
        *l2offset = (uint32_t)len;
        *next_protocol = ntohs(ld16(pkt + len + 12));
        len += 14;
        break;
    default:
        return -1;
    }
    *l2len = (uint32_t)len;
    return 0;
}

/* parse_vlan: get.c:170-182 */
static int parse_vlan(const uint8_t *pkt, uint32_t datalen, uint16_t *next_protocol, uint32_t *l2len)
{
    if ((size_t)datalen < *l2len + 4)
        return -1;
    *next_protocol = ntohs(ld16(pkt + *l2len + 2));
    *l2len += 4;
    return 0;
}

/* parse_metadata: get.c:196-236 */
static int parse_metadata(const uint8_t *pkt, uint32_t datalen, uint16_t *next_protocol, uint32_t *l2len,
                          uint32_t *l2offset, uint32_t *vlan_offset)
{
    for (;;) {
        switch (*next_protocol) {
        case ETHERTYPE_VLAN:
        case ETHERTYPE_Q_IN_Q:
        case ETHERTYPE_8021QINQ:
            if (*vlan_offset == 0)
                *vlan_offset = *l2len;
            if (parse_vlan(pkt, datalen, next_protocol, l2len))
                return -1;
            break;
        case ETHERTYPE_MPLS:
        case ETHERTYPE_MPLS_MULTI:
            if (parse_mpls(pkt, datalen, next_protocol, l2len, l2offset))
                return -1;
            break;
        default:
            return 0;
        }
    }
}

/* get_l2len_protocol, DLT_EN10MB case: get.c:262-380 */
static int get_l2len_protocol(const uint8_t *pkt, uint32_t datalen, uint16_t *protocol, uint32_t *l2len,
                              uint32_t *l2offset, uint32_t *vlan_offset)
{
    if (!datalen)
        return -1;
    *protocol = 0;
    *l2len = 0;
    *l2offset = 0;
    *vlan_offset = 0;
    uint32_t l2_net_off = 14 + *l2offset;
    if (datalen <= l2_net_off + 4)
        return -1;
    uint16_t ether_type = ntohs(ld16(pkt + *l2offset + 12));
    if (parse_metadata(pkt, datalen, &ether_type, &l2_net_off, l2offset, vlan_offset))
        return -1;
    *l2len = l2_net_off;
    if (ether_type >= 1536) {
        *protocol = ether_type;
    } else {
        return -1; /* 802.3 length / unsupported (get.c:367-380) */
    }
    return 0;
}

/* get_l2len: get.c:456-470 (returns 0 on parse failure) */
static int get_l2len(const uint8_t *pkt, int datalen)
{
    uint16_t protocol;
    uint32_t l2offset, vlan_offset, l2len = 0;
    if (get_l2len_protocol(pkt, (uint32_t)datalen, &protocol, &l2len, &l2offset, &vlan_offset) == -1)
        return 0;
    return (int)l2len;
}

/* ------------------------------------------------------------------------- */
/* L3/L4 pointer helpers: get.c:611-853                                      */
/* ------------------------------------------------------------------------- */
/* get_layer4_v4: get.c:611-625 */
static uint8_t *get_layer4_v4(uint8_t *ip, const uint8_t *end)
{
    uint8_t *ptr = ip + ((ip[0] & 0x0f) << 2);
    if (ptr > end)
        return NULL;
    return ptr;
}

static inline bool exthdr_fits(const uint8_t *hdr, const uint8_t *end) /* get.c:636-640 */
{
    return hdr != NULL && hdr + 2 <= end;
}

/* get_ipv6_next: get.c:757-800 */
static uint8_t *get_ipv6_next(uint8_t *exthdr, const uint8_t *end)
{
    if (exthdr + 2 > end)
        return NULL;
    switch (exthdr[0]) {
    case NH_NO_NEXT:
    case NH_ESP:
        return NULL;
    case NH_FRAGMENT: {
        uint8_t *ptr = exthdr + 8;
        if (ptr > end)
            return NULL;
        return ptr;
    }
    case NH_IPV6:
    case NH_ROUTING:
    case NH_DESTOPTS:
    case NH_HBH:
    case NH_AH: {
        uint8_t extlen = (uint8_t)(exthdr[1] * 4 + 8); /* defines.h.in:285, truncated to u8 (get.c:781) */
        if (extlen == 0)
            return NULL;
        uint8_t *ptr = exthdr + extlen;
        if (ptr > end)
            return NULL;
        return ptr;
    }
    default:
        return exthdr;
    }
}

/* get_layer4_v6: get.c:646-750 */
static uint8_t *get_layer4_v6(uint8_t *ip6, const uint8_t *end)
{
    uint8_t *next = ip6 + 40;
    uint8_t *exthdr;
    bool done = false;
    uint8_t proto;
    if (next > end)
        return NULL;
    proto = ip6[6];
    while (!done) {
        switch (proto) {
        case NH_IPV6:
            next = get_layer4_v6(next, end);
            break;
        case NH_AH:
        case NH_ROUTING:
        case NH_DESTOPTS:
        case NH_HBH:
        case NH_FRAGMENT:
            exthdr = get_ipv6_next(next, end);
            if (!exthdr_fits(exthdr, end)) {
                next = NULL;
                done = true;
                break;
            }
            proto = exthdr[0];
            next = exthdr;
            break;
        case NH_ESP:
            next = NULL;
            done = true;
            break;
        default:
            if (proto != ip6[6] && next) {
                if (!exthdr_fits(next, end))
                    return NULL;
                next = next + (next[1] * 4 + 8); /* IPV6_EXTLEN_TO_BYTES, not truncated (get.c:728) */
                if (next > end)
                    return NULL;
            }
            done = true;
        }
        if (next == NULL)
            done = true;
    }
    return next;
}

/* get_ipv6_l4proto: get.c:806-853 */
static uint8_t get_ipv6_l4proto(uint8_t *ip6, const uint8_t *end)
{
    uint8_t *ptr = ip6 + 40;
    uint8_t proto;
    if (ptr > end)
        return NH_NO_NEXT;
    proto = ip6[6];
    for (;;) {
        switch (proto) {
        case NH_NO_NEXT:
        case NH_FRAGMENT:
        case NH_ESP:
            return proto;
        case NH_IPV6:
            return get_ipv6_l4proto(ptr, end);
        case NH_AH:
        case NH_ROUTING:
        case NH_DESTOPTS:
        case NH_HBH: {
            uint8_t *exthdr = get_ipv6_next(ptr, end);
            if (exthdr == NULL || exthdr + 2 > end)
                return NH_NO_NEXT;
            proto = exthdr[0];
            ptr = exthdr;
            break;
        }
        default:
            return proto;
        }
    }
}

/* ------------------------------------------------------------------------- */
/* checksums: src/tcpedit/checksum.c, incremental_checksum.[ch]              */
/* ------------------------------------------------------------------------- */
/* do_checksum_math: checksum.c:175-196 -- sums host-order u16 loads */
static int do_checksum_math(const uint8_t *data, int len)
{
    int sum = 0;
    while (len > 1) {
        sum += ld16(data);
        data += 2;
        len -= 2;
    }
    if (len == 1)
        sum += data[0]; /* pad.b[0]=byte, pad.b[1]=0 read as LE u16 */
    return sum;
}

/* CHECKSUM_CARRY: checksum.h:25 (note: it assigns to its argument) */
#define CHECKSUM_CARRY(x) (x = (x >> 16) + (x & 0xffff), (~(x + (x >> 16)) & 0xffff))

/* do_checksum: checksum.c:34-170 */
static int do_checksum(uint8_t *data, int proto, int len, const uint8_t *end)
{
    bool is_v6 = false;
    int ip_hl;
    int sum = 0;
    if (!data || len <= 0) {
        seterr("length of data must be > 0");
        return TCPEDIT_ERROR;
    }
    if ((data[0] >> 4) == 6) {
        is_v6 = true;
        proto = get_ipv6_l4proto(data, end);
        uint8_t *layer = get_layer4_v6(data, end);
        if (!layer)
            return TCPEDIT_WARN;
        ip_hl = (int)(layer - data);
        len -= (ip_hl - 40);
    } else {
        ip_hl = (data[0] & 0x0f) << 2;
    }
    switch (proto) {
    case IPPROTO_TCP_:
    case IPPROTO_TCP_V6FRAG: {
        if (len < 20)
            return TCPEDIT_WARN;
        uint8_t *tcp = data + ip_hl;
        st16(tcp + 16, 0);
        if (is_v6)
            sum = do_checksum_math(data + 8, 32);
        else
            sum = do_checksum_math(data + 12, 8);
        sum += ntohs((uint16_t)(IPPROTO_TCP_ + len));
        sum += do_checksum_math(tcp, len);
        st16(tcp + 16, (uint16_t)CHECKSUM_CARRY(sum));
        break;
    }
    case IPPROTO_UDP_: {
        if (len < 8)
            return TCPEDIT_WARN;
        uint8_t *udp = data + ip_hl;
        if (ld16(udp + 6) == 0)
            break;
        st16(udp + 6, 0);
        if (is_v6)
            sum = do_checksum_math(data + 8, 32);
        else
            sum = do_checksum_math(data + 12, 8);
        sum += ntohs((uint16_t)(IPPROTO_UDP_ + len));
        sum += do_checksum_math(udp, len);
        st16(udp + 6, (uint16_t)CHECKSUM_CARRY(sum));
        break;
    }
    case IPPROTO_ICMP_: {
        if (len < 4)
            return TCPEDIT_WARN;
        uint8_t *icmp = data + ip_hl;
        st16(icmp + 2, 0);
        if (is_v6) {
            sum = do_checksum_math(data + 8, 32);
            st16(icmp + 2, (uint16_t)CHECKSUM_CARRY(sum));
        }
        sum += do_checksum_math(icmp, len);
        st16(icmp + 2, (uint16_t)CHECKSUM_CARRY(sum));
        break;
    }
    case IPPROTO_ICMP6_: {
        if (len < 8)
            return TCPEDIT_WARN;
        uint8_t *icmp6 = data + ip_hl;
        st16(icmp6 + 2, 0);
        if (is_v6)
            sum = do_checksum_math(data + 8, 32);
        sum += ntohs((uint16_t)(IPPROTO_ICMP6_ + len));
        sum += do_checksum_math(icmp6, len);
        st16(icmp6 + 2, (uint16_t)CHECKSUM_CARRY(sum));
        break;
    }
    default:
        if (!is_v6) {
            st16(data + 10, 0);
            sum = do_checksum_math(data, ip_hl);
            st16(data + 10, (uint16_t)CHECKSUM_CARRY(sum));
        } else {
            return TCPEDIT_WARN;
        }
    }
    return TCPEDIT_OK;
}

/* incremental_checksum.c:30-118 and incremental_checksum.h:46-118 */
static unsigned int do_csum_aligned32(const uint8_t *buff, int len) /* do_csum for a 4-aligned, len%4==0 buffer */
{
    unsigned int result = 0;
    unsigned int carry = 0;
    for (int i = 0; i < len; i += 4) {
        unsigned int w = ld32(buff + i);
        result += carry;
        result += w;
        carry = (w > result);
    }
    result += carry;
    result = (result & 0xffff) + (result >> 16);
    result = (result & 0xffff) + (result >> 16); /* from32to16 */
    result = (result & 0xffff) + (result >> 16);
    return result;
}

static inline uint16_t csum_fold(uint32_t sum)
{
    sum = (sum & 0xffff) + (sum >> 16);
    sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)~sum;
}
static inline uint32_t csum_add(uint32_t csum, uint32_t addend)
{
    uint32_t res = csum + addend;
    return res + (res < addend);
}
static inline uint32_t csum_sub(uint32_t csum, uint32_t addend) { return csum_add(csum, ~addend); }
static inline uint16_t csum16_add(uint16_t csum, uint16_t addend)
{
    uint16_t res = csum;
    res += addend;
    return (uint16_t)(res + (res < addend));
}
static inline uint16_t csum16_sub(uint16_t csum, uint16_t addend) { return csum16_add(csum, (uint16_t)~addend); }

static void csum_replace2(uint8_t *sump, uint16_t from, uint16_t to)
{
    uint16_t sum = ld16(sump);
    st16(sump, (uint16_t)~csum16_add(csum16_sub((uint16_t)~sum, from), to));
}
static void csum_replace4(uint8_t *sump, uint32_t from, uint32_t to)
{
    uint16_t sum = ld16(sump);
    st16(sump, csum_fold(csum_add(csum_sub(~(uint32_t)sum, from), to)));
}
static void csum_replace16(uint8_t *sump, const uint8_t *from, const uint8_t *to)
{
    uint32_t diff[8];
    for (int i = 0; i < 4; i++) {
        diff[i] = ~ld32(from + 4 * i);
        diff[4 + i] = ld32(to + 4 * i);
    }
    uint16_t sum = ld16(sump);
    uint32_t wsum = ~(uint32_t)sum;
    unsigned int result = do_csum_aligned32((const uint8_t *)diff, 32);
    result += wsum; /* csum_partial: incremental_checksum.c:108-118 */
    if (wsum > result)
        result += 1;
    st16(sump, csum_fold(result));
}

/* ------------------------------------------------------------------------- */
/* edit_packet.c                                                             */
/* ------------------------------------------------------------------------- */
static bool is_multicast_ipv4(uint32_t ip) { return (ntohl(ip) & 0xf0000000) == 0xe0000000; } /* :1204 */
static void set_multicast_ipv4(uint32_t *ip) { *ip = htonl((ntohl(*ip) & 0x0fffffff) | 0xe0000000); }
static void set_unicast_ipv4(uint32_t *ip) { *ip = htonl(ntohl(*ip) & 0x7fffffff); }
static bool is_multicast_ipv6(const uint8_t *a) { return a[0] == 0xff; } /* :1229 */

/* fix_ipv4_checksums: edit_packet.c:55-112 */
static int fix_ipv4_checksums(ohdr_t *h, uint8_t *ip, size_t l2len)
{
    int ret1 = 0, ret2, ip_len;
    if (h->caplen < 20 + l2len)
        return TCPEDIT_WARN;
    if ((ip[0] >> 4) != 4) {
        seterr("Invalid packet: Expected IPv4 packet: got %u", ip[0] >> 4);
        return TCPEDIT_ERROR;
    }
    ip_len = (int)ntohs(ld16(ip + 2));
    if (h->caplen == h->len && (htons(ld16(ip + 6)) & (IP_MF | IP_OFFMASK)) == 0) {
        if (ip_len != (int)(h->caplen - l2len))
            return TCPEDIT_WARN;
        ret1 = do_checksum(ip, ip[9], ip_len - ((ip[0] & 0x0f) << 2), ip + h->caplen - l2len);
        if (ret1 < 0)
            return TCPEDIT_ERROR;
    }
    ret2 = do_checksum(ip, IPPROTO_IP_, ip_len, ip + h->caplen - l2len);
    if (ret2 < 0)
        return TCPEDIT_ERROR;
    if (ret1 == TCPEDIT_WARN || ret2 == TCPEDIT_WARN)
        return TCPEDIT_WARN;
    return TCPEDIT_OK;
}

/* ipv6_header_length: edit_packet.c:118-140 */
static int ipv6_header_length(const uint8_t *ip6, size_t pkt_len, size_t l2len)
{
    int offset = 40;
    uint8_t next_header = ip6[6];
    while (2 + offset + l2len < pkt_len) {
        if (next_header != NH_HBH && next_header != NH_ROUTING && next_header != NH_FRAGMENT)
            return offset;
        const uint8_t *nhdr = ip6 + offset;
        next_header = nhdr[0];
        offset += ((nhdr[1] + 1) << 3);
    }
    return -1;
}

/* fix_ipv6_checksums: edit_packet.c:142-189 */
static int fix_ipv6_checksums(ohdr_t *h, uint8_t *ip6, size_t l2len)
{
    int ret = 0;
    if (h->caplen < 40 + l2len)
        return TCPEDIT_WARN;
    if ((ip6[0] >> 4) != 6) {
        seterr("Invalid packet: Expected IPv6 packet: got %u", ip6[0] >> 4);
        return TCPEDIT_ERROR;
    }
    if (h->caplen == h->len) {
        int ip6_len = ipv6_header_length(ip6, h->len, l2len);
        /* compares the raw network-order field with a host int (:167) */
        if ((int)ld16(ip6 + 4) < ip6_len)
            return TCPEDIT_WARN;
        ret = do_checksum(ip6, ip6[6], htons(ld16(ip6 + 4)), ip6 + h->caplen - l2len);
        if (ret < 0)
            return TCPEDIT_ERROR;
    }
    if (ret == TCPEDIT_WARN)
        return TCPEDIT_WARN;
    return TCPEDIT_OK;
}

/* ipv4_l34_csum_replace + ipv4_addr_csum_replace: edit_packet.c:191-296 */
static void ipv4_addr_csum_replace(uint8_t *ip, uint32_t old_ip, uint32_t new_ip, int l3len)
{
    int len = l3len;
    uint8_t *l4;
    if ((size_t)len < 20)
        return;
    csum_replace4(ip + 10, old_ip, new_ip);
    uint8_t protocol = ip[9];
    switch (protocol) {
    case IPPROTO_UDP_:
        l4 = get_layer4_v4(ip, ip + l3len);
        len -= (ip[0] & 0x0f) << 2;
        len -= 8;
        break;
    case IPPROTO_TCP_:
        l4 = get_layer4_v4(ip, ip + l3len);
        len -= (ip[0] & 0x0f) << 2;
        len -= 20;
        break;
    default:
        l4 = NULL;
    }
    if (!l4 || len < 0)
        return;
    if ((htons(ld16(ip + 6)) & IP_OFFMASK) == 0) {
        if (protocol == IPPROTO_TCP_)
            csum_replace4(l4 + 16, old_ip, new_ip);
        else if (ld16(l4 + 6))
            csum_replace4(l4 + 6, old_ip, new_ip);
    }
}

/* ipv6_l34_csum_replace + ipv6_addr_csum_replace: edit_packet.c:222-330 */
static void ipv6_addr_csum_replace(uint8_t *ip6, const uint8_t *old_ip, const uint8_t *new_ip, int l3len)
{
    if ((size_t)l3len < 40)
        return;
    uint8_t protocol = get_ipv6_l4proto(ip6, ip6 + l3len);
    uint8_t *l4;
    switch (protocol) {
    case IPPROTO_UDP_:
    case IPPROTO_TCP_:
    case IPPROTO_ICMP6_:
        l4 = get_layer4_v6(ip6, ip6 + l3len);
        break;
    default:
        l4 = NULL;
    }
    if (!l4)
        return;
    switch (protocol) {
    case IPPROTO_TCP_: csum_replace16(l4 + 16, old_ip, new_ip); break;
    case IPPROTO_UDP_:
        if (ld16(l4 + 6))
            csum_replace16(l4 + 6, old_ip, new_ip);
        break;
    case IPPROTO_ICMP6_: csum_replace16(l4 + 2, old_ip, new_ip); break;
    }
}

/* randomize_ipv4_addr: edit_packet.c:336-357 */
static uint32_t randomize_ipv4_addr(const ocfg_t *c, uint32_t ip)
{
    bool was_multicast = is_multicast_ipv4(ip);
    if (c->skip_broadcast && is_multicast_ipv4(ip))
        return ip;
    uint32_t res_ip = ((ip ^ htonl(c->seed)) - (ip & htonl(c->seed)));
    if (was_multicast && !is_multicast_ipv4(res_ip))
        set_multicast_ipv4(&res_ip);
    else if (!was_multicast && is_multicast_ipv4(res_ip))
        set_unicast_ipv4(&res_ip);
    return res_ip;
}

/* randomize_ipv6_addr: edit_packet.c:359-379 */
static void randomize_ipv6_addr(const ocfg_t *c, uint8_t *addr)
{
    bool was_multicast = is_multicast_ipv6(addr);
    for (int i = 0; i < 4; ++i) {
        uint32_t p = ld32(addr + 4 * i);
        p = ((p ^ htonl(c->seed)) - (p & htonl(c->seed)));
        st32(addr + 4 * i, p);
    }
    if (was_multicast && !is_multicast_ipv6(addr))
        addr[0] = 0xff;
    else if (!was_multicast && is_multicast_ipv6(addr))
        addr[0] = 0xaa;
}

/* fix_ipv4_length / fix_ipv6_length: edit_packet.c:381-413 */
static int fix_ipv4_length(ohdr_t *h, uint8_t *ip, size_t l2len)
{
    int ip_len = (int)ntohs(ld16(ip + 2));
    int ip_len_want = (int)(h->len - l2len);
    if (h->caplen < l2len + 20)
        return -1;
    if ((htons(ld16(ip + 6)) & (IP_MF | IP_OFFMASK)) == 0 && ip_len != ip_len_want) {
        st16(ip + 2, htons((uint16_t)ip_len_want));
        return 1;
    }
    return 0;
}
static int fix_ipv6_length(ohdr_t *h, uint8_t *ip6, size_t l2len)
{
    int ip_len = ntohs(ld16(ip6 + 4));
    int ip_len_want = (int)(h->len - l2len - 40);
    if (h->caplen < l2len + 40)
        return -1;
    if (ip_len != ip_len_want) {
        st16(ip6 + 4, htons((uint16_t)ip_len_want));
        return 1;
    }
    return 0;
}

/* randomize_ipv4: edit_packet.c:420-467 */
static int randomize_ipv4(const ocfg_t *c, ohdr_t *h, uint8_t *ip, int l3len)
{
    if (l3len < (int)(ip[0] & 0x0f) << 2) {
        seterr("Unable to randomize IP header due to packet capture snap length %u", h->caplen);
        return TCPEDIT_ERROR;
    }
    if ((c->skip_broadcast && !is_multicast_ipv4(ld32(ip + 16))) || !c->skip_broadcast) {
        uint32_t old_ip = ld32(ip + 16);
        st32(ip + 16, randomize_ipv4_addr(c, old_ip));
        ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 16), l3len);
    }
    if ((c->skip_broadcast && !is_multicast_ipv4(ld32(ip + 12))) || !c->skip_broadcast) {
        uint32_t old_ip = ld32(ip + 12);
        st32(ip + 12, randomize_ipv4_addr(c, old_ip));
        ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 12), l3len);
    }
    return 0;
}

/* randomize_ipv6: edit_packet.c:469-518 */
static int randomize_ipv6(const ocfg_t *c, ohdr_t *h, uint8_t *ip6, int l3len)
{
    if (l3len < 40) {
        seterr("Unable to randomize IPv6 header due to packet capture snap length %u", h->caplen);
        return TCPEDIT_ERROR;
    }
    if ((c->skip_broadcast && !is_multicast_ipv6(ip6 + 24)) || !c->skip_broadcast) {
        uint8_t old[16];
        memcpy(old, ip6 + 24, 16);
        randomize_ipv6_addr(c, ip6 + 24);
        ipv6_addr_csum_replace(ip6, old, ip6 + 24, l3len);
    }
    if ((c->skip_broadcast && !is_multicast_ipv6(ip6 + 8)) || !c->skip_broadcast) {
        uint8_t old[16];
        memcpy(old, ip6 + 8, 16);
        randomize_ipv6_addr(c, ip6 + 8);
        ipv6_addr_csum_replace(ip6, old, ip6 + 8, l3len);
    }
    return 0;
}

/* untrunc_packet: edit_packet.c:526-621 */
static int untrunc_packet(const ocfg_t *c, ohdr_t *h, uint8_t *packet, uint8_t *ip, uint8_t *ip6)
{
    int l2len;
    int chksum = 1;
    if ((h->caplen == h->len) || (ip == NULL && ip6 == NULL)) {
        if (!c->mtu_truncate)
            return 0;
    }
    /* layer2len(): the encoder plugin's l2len (dlt.c), en10mb.c:917-943 */
    if (h->caplen < 14) {
        l2len = -1;
    } else {
        l2len = get_l2len(packet, (int)h->caplen);
        if (l2len <= 0 || (int)h->caplen < l2len)
            l2len = -1;
    }
    if (l2len < 0) {
        seterr("Non-sensical layer 2 length: %d", l2len);
        return -1;
    }
    if (ip) {
        if ((htons(ld16(ip + 6)) & IP_OFFMASK) != 0) {
            chksum = 0;
        } else if (ip[9] == IPPROTO_UDP_ && (htons(ld16(ip + 6)) & IP_MF) != 0) {
            st16(ip + ((ip[0] & 0x0f) << 2) + 6, 0);
            chksum = 0;
        }
    }
    if (c->fixlen == FIXLEN_PAD) {
        if (h->len > h->caplen) {
            memset(packet + h->caplen, 0, h->len - h->caplen);
            h->caplen = h->len;
        } else if (h->len < h->caplen) {
            seterr("WTF?  Why is your packet larger then the capture len?");
            return -1;
        }
    } else if (c->fixlen == FIXLEN_TRUNC) {
        if (ip && h->len != h->caplen)
            st16(ip + 2, htons((uint16_t)(h->caplen - l2len)));
        h->len = h->caplen;
    } else if (c->mtu_truncate) {
        if (h->len > (uint32_t)(c->mtu + l2len)) {
            h->len = h->caplen = l2len + c->mtu;
            if (ip) {
                st16(ip + 2, htons((uint16_t)c->mtu));
            } else if (ip6) {
                st16(ip6 + 4, htons((uint16_t)(c->mtu - 40)));
            } else {
                chksum = 0;
            }
        }
    } else {
        seterr("Invalid fixlen value: 0x%x", c->fixlen);
        return -1;
    }
    return chksum;
}

/* rewrite_ipv4_ttl: edit_packet.c:627-667 */
static int rewrite_ipv4_ttl(const ocfg_t *c, uint8_t *ip)
{
    if (ip == NULL || c->ttl_mode == TTL_OFF)
        return 0;
    uint16_t oldval = (uint16_t)ip[8];
    switch (c->ttl_mode) {
    case TTL_SET:
        if (ip[8] == c->ttl_value)
            return 0;
        ip[8] = c->ttl_value;
        break;
    case TTL_ADD:
        if (((int)ip[8] + c->ttl_value) > 255)
            ip[8] = 255;
        else
            ip[8] += c->ttl_value;
        break;
    case TTL_SUB:
        if (ip[8] <= c->ttl_value)
            ip[8] = 1;
        else
            ip[8] -= c->ttl_value;
        break;
    }
    uint16_t newval = (uint16_t)ip[8];
    csum_replace2(ip + 10, oldval, newval);
    return 1;
}

/* rewrite_ipv6_hlim: edit_packet.c:673-706 */
static int rewrite_ipv6_hlim(const ocfg_t *c, uint8_t *ip6)
{
    if (ip6 == NULL || c->ttl_mode == TTL_OFF)
        return 0;
    switch (c->ttl_mode) {
    case TTL_SET:
        if (ip6[7] == c->ttl_value)
            return 0;
        ip6[7] = c->ttl_value;
        break;
    case TTL_ADD:
        if (((int)ip6[7] + c->ttl_value) > 255)
            ip6[7] = 255;
        else
            ip6[7] += c->ttl_value;
        break;
    case TTL_SUB:
        if (ip6[7] <= c->ttl_value)
            ip6[7] = 1;
        else
            ip6[7] -= c->ttl_value;
        break;
    }
    return 1;
}

/* ip_in_cidr: cidr.c:425-468 (64-bit unsigned long mask) */
static int ip_in_cidr(const ocidr_t *cidr, uint32_t ip)
{
    if (cidr->family != 4)
        return 0;
    if (cidr->masklen == 0 && cidr->network == 0)
        return 1;
    unsigned long mask = ~0UL;
    mask = mask << (32 - cidr->masklen);
    unsigned long ipaddr = (unsigned long)ntohl(ip) & mask;
    unsigned long network = (unsigned long)htonl(cidr->network) & mask;
    return network == ipaddr;
}

/* ip6_in_cidr: cidr.c:478-529 */
static int ip6_in_cidr(const ocidr_t *cidr, const uint8_t *addr)
{
    uint32_t i, j, k;
    if (cidr->family != 6)
        return 0;
    if (cidr->masklen == 0 && ld32(addr) == 0 && ld32(addr + 4) == 0 && ld32(addr + 8) == 0 && ld32(addr + 12) == 0)
        return 1;
    j = (uint32_t)cidr->masklen / 8;
    for (i = 0; i < j; i++)
        if (addr[i] != cidr->network6[i])
            return 0;
    if ((k = (uint32_t)cidr->masklen % 8) == 0)
        return 1;
    k = (uint32_t)~0 << (8 - k);
    i = addr[j] & k;
    j = cidr->network6[j] & k;
    return i == j;
}

/* remap_ipv4: edit_packet.c:713-746.  A shift by 32 (masklen 0) is masked to
 * 0 by the x86 shl the reference compiles to, so the shift count is &31. */
static uint32_t remap_ipv4(const ocfg_t *c, const ocidr_t *cidr, uint32_t original)
{
    if (cidr->family != 4)
        return 0;
    if (c->skip_broadcast && is_multicast_ipv4(original))
        return original;
    uint32_t mask = 0xffffffffu;
    mask = mask << ((32 - cidr->masklen) & 31);
    uint32_t network = htonl(cidr->network) & mask;
    mask = mask ^ 0xffffffffu;
    uint32_t ipaddr = ntohl(original) & mask;
    return htonl(network ^ ipaddr);
}

/* remap_ipv6: edit_packet.c:748-779.  For masklen%8 != 0 the reference writes
 * addr[addr[j] & k] with shift counts > 31; x86 masks shift counts to 5 bits,
 * which is restated explicitly here. */
static int remap_ipv6(const ocfg_t *c, const ocidr_t *cidr, uint8_t *addr)
{
    uint32_t i, j, k;
    if (cidr->family != 6)
        return 0;
    if (c->skip_broadcast && is_multicast_ipv6(addr))
        return 0;
    j = (uint32_t)cidr->masklen / 8;
    for (i = 0; i < j; i++)
        addr[i] = cidr->network6[i];
    if ((k = (uint32_t)cidr->masklen % 8) == 0)
        return 1;
    k = (uint32_t)~0 << (8 - k);
    i = addr[i] & k;
    {
        uint32_t s1 = (8u - k) & 31u, s2 = k & 31u;
        addr[i] = (uint8_t)((cidr->network6[j] & (0xffu << s1)) | (addr[i] & (0xffu >> s2)));
    }
    return 1;
}

/* rewrite_ipv4l3: edit_packet.c:787-879 */
static int rewrite_ipv4l3(const ocfg_t *c, uint8_t *ip, int dir, int len)
{
    int didsrc = 0, diddst = 0, loop = 1;
    for (int m = 0; m < c->n_srcipmap; m++) {
        if (ip_in_cidr(&c->srcipmap[m].from, ld32(ip + 12))) {
            uint32_t old_ip = ld32(ip + 12);
            st32(ip + 12, remap_ipv4(c, &c->srcipmap[m].to, old_ip));
            ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 12), len);
            break;
        }
    }
    for (int m = 0; m < c->n_dstipmap; m++) {
        if (ip_in_cidr(&c->dstipmap[m].from, ld32(ip + 16))) {
            uint32_t old_ip = ld32(ip + 16);
            st32(ip + 16, remap_ipv4(c, &c->dstipmap[m].to, old_ip));
            ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 16), len);
            break;
        }
    }
    if (c->n_cidrmap1 == 0)
        return 0;
    const ocidrmap_t *l1, *l2;
    int n1, n2, i1 = 0, i2 = 0;
    if (dir == DIR_C2S) {
        l1 = c->cidrmap1; n1 = c->n_cidrmap1;
        l2 = c->cidrmap2; n2 = c->n_cidrmap2;
    } else {
        l1 = c->cidrmap2; n1 = c->n_cidrmap2;
        l2 = c->cidrmap1; n2 = c->n_cidrmap1;
    }
    do {
        if (!diddst && ip_in_cidr(&l2[i2].from, ld32(ip + 16))) {
            uint32_t old_ip = ld32(ip + 16);
            st32(ip + 16, remap_ipv4(c, &l2[i2].to, old_ip));
            ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 16), len);
            diddst = 1;
        }
        if (!didsrc && ip_in_cidr(&l1[i1].from, ld32(ip + 12))) {
            uint32_t old_ip = ld32(ip + 12);
            st32(ip + 12, remap_ipv4(c, &l1[i1].to, old_ip));
            ipv4_addr_csum_replace(ip, old_ip, ld32(ip + 12), len);
            didsrc = 1;
        }
        if (!(diddst && didsrc) && !((i1 + 1 >= n1) && (i2 + 1 >= n2))) {
            if (i1 + 1 < n1)
                i1++;
            if (i2 + 1 < n2)
                i2++;
        } else {
            loop = 0;
        }
    } while (loop);
    return 0;
}

/* rewrite_ipv6l3: edit_packet.c:881-1019 */
static int rewrite_ipv6l3(const ocfg_t *c, uint8_t *ip6, int dir, int l3len)
{
    int didsrc = 0, diddst = 0, loop = 1;
    for (int m = 0; m < c->n_srcipmap; m++) {
        if (ip6_in_cidr(&c->srcipmap[m].from, ip6 + 8)) {
            uint8_t old[16];
            memcpy(old, ip6 + 8, 16);
            remap_ipv6(c, &c->srcipmap[m].to, ip6 + 8);
            ipv6_addr_csum_replace(ip6, old, ip6 + 8, l3len);
            break;
        }
    }
    for (int m = 0; m < c->n_dstipmap; m++) {
        if (ip6_in_cidr(&c->dstipmap[m].from, ip6 + 24)) {
            uint8_t old[16];
            memcpy(old, ip6 + 24, 16);
            remap_ipv6(c, &c->dstipmap[m].to, ip6 + 24);
            ipv6_addr_csum_replace(ip6, old, ip6 + 24, l3len);
            break;
        }
    }
    if (c->n_cidrmap1 != 0) {
        const ocidrmap_t *l1, *l2;
        int n1, n2, i1 = 0, i2 = 0;
        if (dir == DIR_C2S) {
            l1 = c->cidrmap1; n1 = c->n_cidrmap1;
            l2 = c->cidrmap2; n2 = c->n_cidrmap2;
        } else {
            l1 = c->cidrmap2; n1 = c->n_cidrmap2;
            l2 = c->cidrmap1; n2 = c->n_cidrmap1;
        }
        do {
            if (!diddst && ip6_in_cidr(&l2[i2].from, ip6 + 24)) {
                uint8_t old[16];
                memcpy(old, ip6 + 24, 16);
                remap_ipv6(c, &l2[i2].to, ip6 + 24);
                ipv6_addr_csum_replace(ip6, old, ip6 + 24, l3len);
                diddst = 1;
            }
            if (!didsrc && ip6_in_cidr(&l1[i1].from, ip6 + 8)) {
                uint8_t old[16];
                memcpy(old, ip6 + 8, 16);
                remap_ipv6(c, &l1[i1].to, ip6 + 8);
                ipv6_addr_csum_replace(ip6, old, ip6 + 8, l3len);
                didsrc = 1;
            }
            if (!(diddst && didsrc) && !((i1 + 1 >= n1) && (i2 + 1 >= n2))) {
                if (i1 + 1 < n1)
                    i1++;
                if (i2 + 1 < n2)
                    i2++;
            } else {
                loop = 0;
            }
        } while (loop);
    }
    /* ICMPv6 error recursion: edit_packet.c:988-1013 */
    if (l3len > 0) {
        const uint8_t *end = ip6 + l3len;
        uint8_t l4proto = get_ipv6_l4proto(ip6, end);
        if (l4proto == IPPROTO_ICMP6_) {
            uint8_t *icmp6 = get_layer4_v6(ip6, end);
            if (icmp6 != NULL && icmp6 + 8 <= end) {
                switch (icmp6[0]) {
                case 1: case 2: case 3: case 4: {
                    uint8_t *emb = icmp6 + 8;
                    int emb_len = (int)(end - emb);
                    if (emb_len >= 40 && (emb[0] >> 4) == 6)
                        rewrite_ipv6l3(c, emb, dir, emb_len);
                    break;
                }
                default:
                    break;
                }
            }
        }
    }
    return 0;
}

/* randomize_iparp: edit_packet.c:1025-1083 */
static int randomize_iparp(const ocfg_t *c, ohdr_t *h, uint8_t *pkt, int l3len)
{
    if (l3len < 8) {
        seterr("Unable to randomize ARP packet due to packet capture snap length %u", h->caplen);
        return TCPEDIT_ERROR;
    }
    int l2len = get_l2len(pkt, (int)h->caplen);
    uint8_t *arp = pkt + l2len;
    uint16_t op = ntohs(ld16(arp + 6));
    if (ntohs(ld16(arp + 2)) == ETHERTYPE_IP && (op == 1 || op == 2)) {
        uint8_t *add_hdr = arp + 8 + arp[4];
        st32(add_hdr, randomize_ipv4_addr(c, ld32(add_hdr)));
        add_hdr += arp[5] + arp[4];
        st32(add_hdr, randomize_ipv4_addr(c, ld32(add_hdr)));
    }
    return 1;
}

/* rewrite_iparp: edit_packet.c:1093-1198 */
static int rewrite_iparp(const ocfg_t *c, uint8_t *arp, int dir)
{
    const ocidrmap_t *l1 = NULL, *l2 = NULL;
    int n1 = 0, n2 = 0, i1 = 0, i2 = 0;
    int didsrc = 0, diddst = 0, loop = 1;
    if (dir == DIR_C2S) {
        l1 = c->cidrmap1; n1 = c->n_cidrmap1;
        l2 = c->cidrmap2; n2 = c->n_cidrmap2;
    } else if (dir == DIR_S2C) {
        l1 = c->cidrmap2; n1 = c->n_cidrmap2;
        l2 = c->cidrmap1; n2 = c->n_cidrmap1;
    }
    if (n1 == 0 || n2 == 0)
        return 0;
    uint16_t op = ntohs(ld16(arp + 6));
    if (ntohs(ld16(arp + 2)) == ETHERTYPE_IP && (op == 1 || op == 2)) {
        uint8_t *ip1 = arp + 8 + arp[4];
        uint8_t *ip2 = ip1 + arp[5] + arp[4];
        do {
            if (op == 1) {
                if (!diddst && ip_in_cidr(&l2[i2].from, ld32(ip1))) {
                    st32(ip1, remap_ipv4(c, &l2[i2].to, ld32(ip1)));
                    diddst = 1;
                }
                if (!didsrc && ip_in_cidr(&l1[i1].from, ld32(ip2))) {
                    st32(ip2, remap_ipv4(c, &l1[i1].to, ld32(ip2)));
                    didsrc = 1;
                }
            } else {
                if (!diddst && ip_in_cidr(&l2[i2].from, ld32(ip2))) {
                    st32(ip2, remap_ipv4(c, &l2[i2].to, ld32(ip2)));
                    diddst = 1;
                }
                if (!didsrc && ip_in_cidr(&l1[i1].from, ld32(ip1))) {
                    st32(ip1, remap_ipv4(c, &l1[i1].to, ld32(ip1)));
                    didsrc = 1;
                }
            }
            if (!(diddst && didsrc) && !((i1 + 1 >= n1) && (i2 + 1 >= n2))) {
                if (i1 + 1 < n1)
                    i1++;
                if (i2 + 1 < n2)
                    i2++;
            } else {
                loop = 0;
            }
        } while (loop);
    } else {
        g_warn_count++; /* warn("ARP packet isn't for IPv4!...") edit_packet.c:1194 */
    }
    return didsrc + diddst;
}

/* ------------------------------------------------------------------------- */
/* portmap.c:239-372, rewrite_sequence.c:37-92                               */
/* ------------------------------------------------------------------------- */
static long map_port(const ocfg_t *c, long port) /* portmap.c:239-260 */
{
    for (int i = 0; i < c->n_portmap; i++)
        if (c->portmap[i].from == port)
            return c->portmap[i].to;
    return port;
}

static int rewrite_ports(const ocfg_t *c, uint8_t protocol, uint8_t *l4, int l4len) /* portmap.c:267-330 */
{
    uint16_t newport;
    if (protocol == IPPROTO_TCP_) {
        if (l4len < 20)
            return TCPEDIT_WARN;
        newport = (uint16_t)map_port(c, ld16(l4 + 2));
        if (newport != ld16(l4 + 2)) {
            csum_replace2(l4 + 16, ld16(l4 + 2), newport);
            st16(l4 + 2, newport);
        }
        newport = (uint16_t)map_port(c, ld16(l4));
        if (newport != ld16(l4)) {
            csum_replace2(l4 + 16, ld16(l4), newport);
            st16(l4, newport);
        }
    } else if (protocol == IPPROTO_UDP_) {
        if (l4len < 8)
            return TCPEDIT_WARN;
        newport = (uint16_t)map_port(c, ld16(l4 + 2));
        if (newport != ld16(l4 + 2)) {
            if (ld16(l4 + 6))
                csum_replace2(l4 + 6, ld16(l4 + 2), newport);
            st16(l4 + 2, newport);
        }
        newport = (uint16_t)map_port(c, ld16(l4));
        if (newport != ld16(l4)) {
            if (ld16(l4 + 6))
                csum_replace2(l4 + 6, ld16(l4), newport);
            st16(l4, newport);
        }
    }
    return 0;
}

static int rewrite_ipv4_ports(const ocfg_t *c, uint8_t *ip, int l3len) /* portmap.c:332-351 */
{
    if (ip[9] == IPPROTO_TCP_ || ip[9] == IPPROTO_UDP_) {
        uint8_t *l4 = get_layer4_v4(ip, ip + l3len);
        if (l4)
            return rewrite_ports(c, ip[9], l4, l3len - (int)(l4 - ip));
        return TCPEDIT_WARN;
    }
    return 0;
}

static int rewrite_ipv6_ports(const ocfg_t *c, uint8_t *ip6, int l3len) /* portmap.c:353-372 */
{
    if (ip6[6] == IPPROTO_TCP_ || ip6[6] == IPPROTO_UDP_) {
        uint8_t *l4 = get_layer4_v6(ip6, ip6 + l3len);
        if (l4)
            return rewrite_ports(c, ip6[6], l4, l3len - (int)(l4 - ip6));
        return TCPEDIT_WARN;
    }
    return 0;
}

static int rewrite_seqs(const ocfg_t *c, uint8_t *tcp) /* rewrite_sequence.c:37-55 */
{
    uint32_t newnum = ntohl(ld32(tcp + 4)) + c->tcp_sequence_adjust;
    csum_replace4(tcp + 16, ld32(tcp + 4), htonl(newnum));
    st32(tcp + 4, htonl(newnum));
    if (!((tcp[13] & TH_SYN) && !(tcp[13] & TH_ACK))) {
        newnum = ntohl(ld32(tcp + 8)) + c->tcp_sequence_adjust;
        csum_replace4(tcp + 16, ld32(tcp + 8), htonl(newnum));
        st32(tcp + 8, htonl(newnum));
    }
    return 0;
}

static int rewrite_ipv4_tcp_sequence(const ocfg_t *c, uint8_t *ip, int l3len) /* rewrite_sequence.c:57-74 */
{
    if (ip[9] == IPPROTO_TCP_) {
        uint8_t *tcp = get_layer4_v4(ip, ip + l3len);
        if (!tcp)
            return TCPEDIT_WARN;
        return rewrite_seqs(c, tcp);
    }
    return 0;
}

static int rewrite_ipv6_tcp_sequence(const ocfg_t *c, uint8_t *ip6, int l3len) /* rewrite_sequence.c:76-92 */
{
    if (ip6[6] == IPPROTO_TCP_) {
        uint8_t *tcp = get_layer4_v6(ip6, ip6 + l3len);
        if (!tcp)
            return TCPEDIT_WARN;
        return rewrite_seqs(c, tcp);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* DLT_EN10MB plugin: plugins/dlt_en10mb/en10mb.c, plugins/ethernet.c        */
/* ------------------------------------------------------------------------- */
static int is_unicast_ethernet(const uint8_t *e) /* ethernet.c:30-57 */
{
    static const uint8_t bcast[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    static const uint8_t v4m[3] = {0x01, 0x00, 0x5e};
    static const uint8_t v6m[2] = {0x33, 0x33};
    static const uint8_t vrrp4[5] = {0x00, 0x00, 0x50, 0x00, 0x01}; /* defines.h.in:226 */
    static const uint8_t vrrp6[5] = {0x00, 0x00, 0x50, 0x00, 0x02}; /* defines.h.in:227 */
    if (memcmp(e, bcast, 6) == 0)
        return 0;
    if (memcmp(e, v4m, 3) == 0)
        return 0;
    if (memcmp(e, v6m, 2) == 0)
        return 0;
    if (memcmp(e, vrrp4, 5) == 0 || memcmp(e, vrrp6, 5) == 0)
        return 0;
    return 1;
}

/* dlt_en10mb_l2len: en10mb.c:917-943 */
static int en10mb_l2len(const uint8_t *pkt, int pktlen)
{
    if (pktlen < 14)
        return -1;
    int l2len = get_l2len(pkt, pktlen);
    if (l2len > 0) {
        if (pktlen < l2len)
            return -1;
        return l2len;
    }
    return -1;
}

/* dlt_en10mb_proto: en10mb.c:741-762 (returns the ethertype in network order) */
static int en10mb_proto(const uint8_t *pkt, int pktlen)
{
    uint16_t ether_type;
    uint32_t l2offset, l2len, vlan_offset;
    if (pktlen < 14)
        return TCPEDIT_ERROR;
    if (get_l2len_protocol(pkt, (uint32_t)pktlen, &ether_type, &l2len, &l2offset, &vlan_offset) == -1)
        return TCPEDIT_ERROR;
    return htons(ether_type);
}

/* dlt_en10mb_decode: en10mb.c:402-473 */
static int en10mb_decode(ostate_t *s, const uint8_t *pkt, int pktlen)
{
    uint16_t protcol;
    uint32_t l2offset, l2len, vlan_offset;
    uint32_t pkt_len = (uint32_t)pktlen;
    if (get_l2len_protocol(pkt, pkt_len, &protcol, &l2len, &l2offset, &vlan_offset) == -1)
        return TCPEDIT_ERROR;
    if (pkt_len < 14 + l2offset)
        return TCPEDIT_ERROR;
    const uint8_t *eth = pkt + l2offset;
    protcol = ntohs(ld16(eth + 12));
    memcpy(s->dstaddr, eth, 6);
    memcpy(s->srcaddr, eth + 6, 6);
    s->proto_vlan_tag = ntohs(ld16(eth + 12));
    if (vlan_offset != 0) {
        if (vlan_offset == l2offset + 14) {
            if (pkt_len < vlan_offset + 4)
                return TCPEDIT_ERROR;
            uint16_t tci = htons(ld16(pkt + vlan_offset));
            s->vlan = 1;
            s->vlan_offset = vlan_offset;
            s->vlan_proto = ntohs(ld16(pkt + vlan_offset + 2));
            s->vlan_tag = tci & VIDMASK;
            s->vlan_pri = tci & PRIMASK;
            s->vlan_cfi = tci & CFIMASK;
        } else {
            return TCPEDIT_ERROR;
        }
    } else {
        s->vlan = 0;
        s->vlan_offset = l2offset + 14;
        s->vlan_proto = protcol;
    }
    s->proto = ntohs(protcol);
    s->l2offset = (int)l2offset;
    s->l2len = (int)l2len;
    return TCPEDIT_OK;
}

/* ---- the other decoders (src/tcpedit/plugins/dlt_*): plugin_proto and plugin_decode ---- */
#define ARPHRD_ETHER 1       /* linuxsll_types.h:56 */
#define ARPHRD_LOOPBACK 772

/* dlt_null_proto: null.c:206-236 (DLT_NULL and DLT_LOOP): the address family in either
   byte order; PF_INET6 is 10 here, and the BSDs' 24/28/30 are taken too */
static int null_proto(const uint8_t *pkt, int pktlen)
{
    if (pktlen < 4)
        return TCPEDIT_ERROR;
    const uint32_t af = ld32(pkt), saf = __builtin_bswap32(af);
    if (af == 2 || saf == 2)
        return htons(ETHERTYPE_IP);
    if (af == 10 || saf == 10 || af == 24 || saf == 24 || af == 28 || saf == 28 || af == 30 || saf == 30)
        return htons(ETHERTYPE_IP6);
    seterr("Unsupported DLT_NULL/DLT_LOOP PF_ type: 0x%04x", af);
    return TCPEDIT_ERROR;
}

/* dlt_raw_proto: raw.c:206-231 (the IP version nibble) */
static int raw_proto(const uint8_t *pkt, int pktlen)
{
    if (pktlen < 20)
        return TCPEDIT_ERROR;
    if ((pkt[0] >> 4) == 4)
        return htons(ETHERTYPE_IP);
    if ((pkt[0] >> 4) == 6)
        return htons(ETHERTYPE_IP6);
    seterr("Unsupported DLT_RAW packet: doesn't look like IPv4 or IPv6");
    return TCPEDIT_ERROR;
}

/* ---- DLT_IEEE802_11 (plugins/dlt_ieee80211/ieee80211.c, ieee80211_hdr.c).  The frame
   control word is read with ntohs, so the masks of ieee80211_types.h:33-76 apply to
   (byte0 << 8 | byte1): type/subtype in the high byte, the DS/WEP flags in the low one. */
#define I80211_FC_TYPE_MASK 0x0F00
#define I80211_FC_TYPE_DATA 0x0800
#define I80211_FC_SUBTYPE_MASK 0xF000
#define I80211_FC_SUBTYPE_QOS 0x8000
#define I80211_FC_SUBTYPE_NULL 0xC000
#define I80211_FC_WEP_MASK 0x0040
#define I80211_USE_4(fc) (((fc)&3) == 3) /* ieee80211_USE_4: TO_DS and FROM_DS */

static uint16_t i80211_fc(const uint8_t *pkt) { return (uint16_t)(pkt[0] << 8 | pkt[1]); }

/* dlt_ieee80211_l2len: ieee80211.c:333-371 (0, not -1, for a short frame) */
static int i80211_l2len(const uint8_t *pkt, int pktlen)
{
    if (pktlen < 2)
        return 0;
    const uint16_t fc = i80211_fc(pkt);
    int hdrlen = I80211_USE_4(fc) ? 30 : 24; /* ieee80211_addr4_hdr_t / ieee80211_hdr_t */
    if ((fc & I80211_FC_SUBTYPE_QOS) == I80211_FC_SUBTYPE_QOS)
        hdrlen += 2;
    if (pktlen >= hdrlen + 8) /* struct tcpr_802_2snap_hdr: 8 bytes, tcpr_802_2_hdr: 3 */
        hdrlen += pkt[hdrlen] == 0xAA && pkt[hdrlen + 1] == 0xAA ? 8 : 3;
    if (pktlen < hdrlen)
        return 0;
    return hdrlen;
}

/* ieee80211_is_data: ieee80211_hdr.c:36-92 */
static int i80211_is_data(const uint8_t *pkt, int pktlen)
{
    if (pktlen <= 24)
        return 0;
    const uint16_t fc = i80211_fc(pkt);
    if ((fc & I80211_FC_SUBTYPE_MASK) == I80211_FC_SUBTYPE_NULL)
        return 1;
    if ((fc & I80211_FC_TYPE_MASK) == I80211_FC_TYPE_DATA)
        return 1;
    int hdrlen = (fc & I80211_FC_SUBTYPE_MASK) >= I80211_FC_SUBTYPE_QOS ? 2 : 0;
    hdrlen += I80211_USE_4(fc) ? 30 : 24;
    if (pktlen < hdrlen + 8)
        return 0;
    return pkt[hdrlen] == 0xAA && pkt[hdrlen + 1] == 0xAA;
}

/* ieee80211_get_src / ieee80211_get_dst: ieee80211_hdr.c:120-184 (addr1 at 4, addr2 at 10,
   addr3 at 16, addr4 at 24) */
static const uint8_t *i80211_src(const uint8_t *pkt)
{
    const uint16_t fc = i80211_fc(pkt);
    if (I80211_USE_4(fc))
        return pkt + 24;
    return (fc & 3) == 2 ? pkt + 16 : pkt + 10; /* FROM_DS: addr3; TO_DS or neither: addr2 */
}
static const uint8_t *i80211_dst(const uint8_t *pkt)
{
    const uint16_t fc = i80211_fc(pkt);
    if (I80211_USE_4(fc))
        return pkt + 16;
    return (fc & 3) == 2 ? pkt + 4 : pkt + 16; /* FROM_DS: addr1; TO_DS or neither: addr3 */
}

/* dlt_ieee80211_proto: ieee80211.c:246-291.  The SNAP header is read at the computed offset
   whatever the captured length (past it: the static buffer's bytes). */
static int i80211_proto(const uint8_t *pkt, int pktlen)
{
    const int l2len = i80211_l2len(pkt, pktlen);
    if (pktlen < l2len)
        return TCPEDIT_ERROR;
    const uint16_t fc = i80211_fc(pkt);
    if ((fc & I80211_FC_TYPE_MASK) != I80211_FC_TYPE_DATA)
        return TCPEDIT_SOFT_ERROR;
    int hdrlen = (fc & I80211_FC_SUBTYPE_QOS) == I80211_FC_SUBTYPE_QOS ? 2 : 0;
    hdrlen += I80211_USE_4(fc) ? 30 : 24;
    if (pkt[hdrlen] == 0xAA && pkt[hdrlen + 1] == 0xAA)
        return ld16(pkt + hdrlen + 6); /* snap_type, network order */
    return TCPEDIT_SOFT_ERROR;
}

/* dlt_ieee80211_decode: ieee80211.c:184-224 */
static int i80211_decode(ostate_t *s, const uint8_t *pkt, int pktlen)
{
    const int l2len = i80211_l2len(pkt, pktlen);
    if (pktlen < l2len)
        return TCPEDIT_ERROR;
    if (!i80211_is_data(pkt, pktlen)) {
        seterr("Packet is not a normal 802.11 data frame");
        return TCPEDIT_SOFT_ERROR;
    }
    if (pktlen >= 24 && (i80211_fc(pkt) & I80211_FC_WEP_MASK) == I80211_FC_WEP_MASK) { /* is_encrypted */
        seterr("Packet is encrypted.  Unable to decode frame.");
        return TCPEDIT_SOFT_ERROR;
    }
    s->l2len = l2len;
    s->l2offset = 0;
    memcpy(s->srcaddr, i80211_src(pkt), 6);
    memcpy(s->dstaddr, i80211_dst(pkt), 6);
    s->proto = (uint16_t)i80211_proto(pkt, pktlen);
    return TCPEDIT_OK;
}

/* ---- DLT_JUNIPER_ETHER (plugins/dlt_jnpr_ether/jnpr_ether.c): a 6-byte header {magic
   4d 47 43, options, extension length (BE)}, TLV extensions, then an Ethernet frame that
   an en10mb sub-decoder decodes.  tcpedit_dlt_copy_decoder_state (dlt_utils.c:249-271)
   hands the sub-decoder's addresses, proto and -- by pointer -- its en10mb extra (the
   inner frame's VLAN fields; dst_modified lives there too) to the encoder, and adds its
   l2len; ctx->l2offset stays 0. */
#define JNPR_HEADER_LEN 6
/* dlt_jnpr_ether_proto: jnpr_ether.c:310-345 */
static int jnpr_proto(const uint8_t *pkt, int pktlen)
{
    if (pktlen < JNPR_HEADER_LEN)
        return TCPEDIT_ERROR;
    if ((pkt[3] & 0x80) != 0x80) /* JUNIPER_ETHER_L2PRESENT */
        return TCPEDIT_ERROR;
    const int hl = (pkt[4] << 8 | pkt[5]) + JNPR_HEADER_LEN;
    if (hl > pktlen)
        return TCPEDIT_ERROR;
    return en10mb_proto(pkt + hl, pktlen - hl);
}
/* dlt_jnpr_ether_decode: jnpr_ether.c:201-282.  A frame whose extensions do not say
   Ethernet (media type 1, encapsulation 14) is a TCPEDIT_WARN: the encoder then runs on
   the previous frame's decoded state with this frame's Juniper header length. */
static int jnpr_decode(ostate_t *s, const uint8_t *pkt, int pktlen)
{
    if (pktlen < JNPR_HEADER_LEN)
        return TCPEDIT_ERROR;
    if (pkt[0] != 0x4d || pkt[1] != 0x47 || pkt[2] != 0x43) {
        seterr("Invalid magic 0x%02X%02X%02X", pkt[0], pkt[1], pkt[2]);
        return TCPEDIT_ERROR;
    }
    if ((pkt[3] & 0x80) != 0x80) {
        seterr("Frame is missing L2 Header: %x", pkt[3]);
        return TCPEDIT_ERROR;
    }
    const int hl = (pkt[4] << 8 | pkt[5]) + JNPR_HEADER_LEN;
    if (pktlen < hl + 14) {
        seterr("Frame is too short! %d < %d", pktlen, hl + 14);
        return TCPEDIT_ERROR;
    }
    s->l2len = hl;
    s->l2offset = 0;
    int ext = JNPR_HEADER_LEN, dlt = 0, encap = 0;
    while (ext < hl - 2) {
        const int ext_len = pkt[ext + 1];
        if (pkt[ext] == 3) /* JUNIPER_ETHER_EXT_MEDIA_TYPE */
            dlt = pkt[ext + 2];
        else if (pkt[ext] == 6) /* JUNIPER_ETHER_EXT_ENCAPSULATION */
            encap = pkt[ext + 2];
        if (dlt != 0 && encap != 0)
            break;
        ext += ext_len + 2;
    }
    if (ext > hl) {
        seterr("Extension to long! %d", ext - hl);
        return TCPEDIT_ERROR;
    }
    if (dlt != 1 || encap != 14) {
        seterr("packet DLT %d and encapsulation type %u not supported", dlt, encap);
        return TCPEDIT_WARN;
    }
    /* the sub-decoder: an en10mb context of its own (config->subctx, jnpr_ether.c:135-136,276)
       whose state is copied into ours only after a whole decode (:280, dlt_utils.c:249-271:
       addresses, proto, the extra by pointer, the l2lens added; not its l2offset) -- a decode
       that fails part-way leaves ours as the last whole one left it, which is what a later
       TCPEDIT_WARN frame encodes with.  Until the first whole decode the encoder's extra is
       our own zeroed one; from it on it is the sub-decoder's, whose dst_modified/src_modified
       no encode has written yet (en10mb_decode never writes them). */
    ostate_t sub = *s;
    if (en10mb_decode(&sub, pkt + hl, pktlen - hl) == TCPEDIT_ERROR)
        return TCPEDIT_ERROR;
    memcpy(s->dstaddr, sub.dstaddr, 6);
    memcpy(s->srcaddr, sub.srcaddr, 6);
    s->proto = sub.proto;
    s->vlan = sub.vlan;
    s->vlan_offset = sub.vlan_offset;
    s->vlan_tag = sub.vlan_tag;
    s->vlan_pri = sub.vlan_pri;
    s->vlan_cfi = sub.vlan_cfi;
    s->vlan_proto = sub.vlan_proto;
    if (!s->jnpr_sub) {
        s->jnpr_sub = true;
        s->dst_modified = s->src_modified = false;
    }
    s->l2len = hl + sub.l2len;
    s->l2offset = 0;
    return TCPEDIT_OK;
}

/* the decoder's proto (tcpedit_dlt_proto on the source DLT, tcpedit.c:96) */
static int decoder_proto(const ocfg_t *c, const uint8_t *pkt, int pktlen)
{
    switch (c->decoder) {
    case DEC_JNPR:
        return jnpr_proto(pkt, pktlen);
    case DEC_80211:
        return i80211_proto(pkt, pktlen);
    case DEC_RADIOTAP: { /* radiotap.c:134-155 */
        if (pktlen < 8) /* sizeof(radiotap_hdr_t) */
            return TCPEDIT_ERROR;
        const int radiolen = pkt[2] | pkt[3] << 8; /* it_len, little endian */
        if (radiolen > pktlen)
            return TCPEDIT_ERROR;
        /* dlt_radiotap_get_80211 (radiotap.c:344-364) copies the 802.11 frame into its
           extra buffer only when it is at least MAXPACKET bytes long, which no record is:
           the 802.11 proto reads the extra's zeros -- frame control 0, not a data frame */
        return TCPEDIT_SOFT_ERROR;
    }
    case DEC_SLL: /* linuxsll.c:213-226 */
        return pktlen < 16 ? TCPEDIT_ERROR : ld16(pkt + 14);
    case DEC_SLL2: /* linuxsll2.c:226-238 */
        return pktlen < 20 ? TCPEDIT_ERROR : ld16(pkt);
    case DEC_RAW:
        return raw_proto(pkt, pktlen);
    case DEC_NULL:
        return null_proto(pkt, pktlen);
    case DEC_PPP: /* pppserial.c:257-281: the ethertype in host order, so tcpedit.c:123,149 never match it */
        if (pktlen < 4)
            return TCPEDIT_ERROR;
        return ntohs(ld16(pkt + 2)) == 0x0021 ? ETHERTYPE_IP : TCPEDIT_SOFT_ERROR;
    case DEC_CHDLC: /* hdlc.c:299-311 */
        return pktlen < 4 ? TCPEDIT_ERROR : ld16(pkt + 2);
    default:
        return en10mb_proto(pkt, pktlen);
    }
}

/* the decoder (plugin_decode): l2len, proto and, for the Linux cooked headers, the source
   address.  None of them touches the en10mb extra fields (vlan, vlan_offset, vlan_proto,
   dst_modified), which keep their zeroed start: the decoder's extra buffer (MAXPACKET
   bytes) is larger than en10mb_extra_t, so en10mb's init keeps it (en10mb.c:100-110) */
static int decoder_decode(const ocfg_t *c, ostate_t *s, const uint8_t *pkt, int pktlen)
{
    switch (c->decoder) {
    case DEC_SLL:  /* linuxsll.c:170-194 */
    case DEC_SLL2: /* linuxsll2.c:181-205 */
    {
        const int sll = c->decoder == DEC_SLL, hl = sll ? 16 : 20;
        if (pktlen < hl)
            return TCPEDIT_ERROR;
        s->proto = ld16(pkt + (sll ? 14 : 0));
        s->l2len = hl;
        const int type = ntohs(ld16(pkt + (sll ? 2 : 8)));
        if (type != ARPHRD_ETHER && type != ARPHRD_LOOPBACK) {
            seterr("DLT_LINUX_SLL pcap's must contain only ethernet or loopback packets");
            return TCPEDIT_ERROR;
        }
        memcpy(s->srcaddr, pkt + (sll ? 6 : 12), 6);
        return TCPEDIT_OK;
    }
    case DEC_RAW: { /* raw.c:170-190 */
        if (pktlen == 0)
            return TCPEDIT_ERROR;
        const int p = raw_proto(pkt, pktlen);
        if (p == TCPEDIT_ERROR)
            return TCPEDIT_ERROR;
        s->proto = (uint16_t)p;
        s->l2len = 0;
        return TCPEDIT_OK;
    }
    case DEC_NULL: { /* null.c:171-187 */
        const int p = null_proto(pkt, pktlen);
        if (p == TCPEDIT_ERROR)
            return TCPEDIT_ERROR;
        s->proto = (uint16_t)p;
        s->l2len = 4;
        return TCPEDIT_OK;
    }
    case DEC_PPP: /* pppserial.c:196-231 */
        if (pktlen < 4)
            return TCPEDIT_ERROR;
        s->proto = ntohs(ld16(pkt + 2)) == 0x0021 ? htons(ETHERTYPE_IP) : ld16(pkt + 2);
        s->l2len = 4;
        return TCPEDIT_OK;
    case DEC_CHDLC: /* hdlc.c:192-218 (its address/control extras are never marked filled) */
        if (pktlen < 4)
            return TCPEDIT_ERROR;
        s->proto = ld16(pkt + 2);
        s->l2len = 4;
        return TCPEDIT_OK;
    case DEC_JNPR:
        return jnpr_decode(s, pkt, pktlen);
    case DEC_80211:
        return i80211_decode(s, pkt, pktlen);
    case DEC_RADIOTAP: /* (its proto never lets a record get here) */
        return TCPEDIT_ERROR;
    default:
        return en10mb_decode(s, pkt, pktlen);
    }
}

/* dlt_en10mb_encode: en10mb.c:479-736 (en10mb decoder -> en10mb encoder) */
static int en10mb_encode(const ocfg_t *c, ostate_t *s, uint8_t *packet, int pktlen, int dir)
{
    uint32_t newl2len = 0, oldl2len = 0;
    if (pktlen < 14)
        return TCPEDIT_ERROR;
    if (c->vlan == VLAN_ADD && !s->vlan && c->vlan_tag == 65535) {
        seterr("Non-VLAN tagged packet requires --enet-vlan-tag");
        return TCPEDIT_ERROR;
    }
    if (c->decoder == DEC_EN10MB) {
        switch (c->vlan) {
        case VLAN_ADD:
            oldl2len = s->vlan_offset;
            newl2len = s->vlan_offset + 4;
            break;
        case VLAN_DEL:
            if (s->vlan) {
                oldl2len = s->vlan_offset + 4;
                newl2len = s->vlan_offset;
            }
            break;
        case VLAN_OFF:
            if (s->vlan) {
                oldl2len = s->vlan_offset;
                newl2len = s->vlan_offset;
            }
            break;
        }
    } else { /* another DLT -> ethernet (en10mb.c:544-548) */
        newl2len = c->vlan == VLAN_ADD ? 18 : 14;
        oldl2len = (uint32_t)s->l2len;
    }
    if ((uint32_t)pktlen < newl2len || pktlen + newl2len - s->l2len > MAXPACKET)
        return TCPEDIT_ERROR;
    if (pktlen < s->l2len)
        return TCPEDIT_ERROR;
    if (newl2len > 0 && newl2len != oldl2len) {
        if (pktlen + (newl2len - oldl2len) > MAXPACKET)
            return TCPEDIT_ERROR;
        memmove(packet + newl2len, packet + oldl2len, pktlen - oldl2len);
    }
    pktlen += (int)(newl2len - oldl2len);
    uint8_t *eth = packet + s->l2offset;
    uint8_t *dhost = eth, *shost = eth + 6;
    const bool l2skip = c->l2_skip_broadcast;
    /* the decoder's address type (plugin_l2addr_type): ETHERNET for en10mb and the Linux
       cooked headers, which have a source address (the destination stays as the zeroed
       context left it); none for the others (en10mb.c:586-659) */
    const bool eth_addr = c->decoder == DEC_EN10MB || c->decoder == DEC_SLL || c->decoder == DEC_SLL2 ||
                          c->decoder == DEC_JNPR || c->decoder == DEC_80211 || c->decoder == DEC_RADIOTAP;
    if (dir == DIR_C2S || dir == DIR_S2C) {
        const bool c2s = dir == DIR_C2S;
        const int sm = c2s ? MASK_SMAC1 : MASK_SMAC2, dm = c2s ? MASK_DMAC1 : MASK_DMAC2;
        if (c->mac_mask & sm) {
            if ((eth_addr && ((l2skip && is_unicast_ethernet(s->srcaddr)) || !l2skip)) || !eth_addr)
                memcpy(shost, c2s ? c->intf1_smac : c->intf2_smac, 6);
            else
                memcpy(shost, s->srcaddr, 6);
        } else if (eth_addr) {
            if (c2s)
                s->src_modified = memcmp(shost, s->srcaddr, 6) != 0;
            memcpy(shost, s->srcaddr, 6);
        } else {
            seterr("Please provide a source address");
            return TCPEDIT_ERROR;
        }
        if (c->mac_mask & dm) {
            if ((eth_addr && ((l2skip && is_unicast_ethernet(s->dstaddr)) || !l2skip)) || !eth_addr)
                memcpy(dhost, c2s ? c->intf1_dmac : c->intf2_dmac, 6);
            else
                memcpy(dhost, s->dstaddr, 6);
        } else if (eth_addr) {
            if (c2s) /* (S2C leaves it: the last C2S packet's value carries over) */
                s->dst_modified = memcmp(dhost, s->dstaddr, 6) != 0;
            memcpy(dhost, s->dstaddr, 6);
        } else {
            seterr("Please provide a destination address");
            return TCPEDIT_ERROR;
        }
    } else {
        seterr("Encoders only support C2S or C2S!");
        return TCPEDIT_ERROR;
    }
    for (int e = 0; e < c->n_subs; e++) {
        if (!memcmp(dhost, c->subs[e][0], 6))
            memcpy(dhost, c->subs[e][1], 6);
        if (!memcmp(shost, c->subs[e][0], 6))
            memcpy(shost, c->subs[e][1], 6);
    }
    if (c->random_set) {
        int unicast_src = is_unicast_ethernet(shost);
        int unicast_dst = is_unicast_ethernet(dhost);
        for (int i = c->random_keep; i < 6; i++) {
            int ms = c->random_mask[i] * unicast_src, md = c->random_mask[i] * unicast_dst;
            shost[i] = (uint8_t)((shost[i] ^ ms) - (shost[i] & ms)); /* MAC_MASK_APPLY en10mb.h:29-30 */
            dhost[i] = (uint8_t)((dhost[i] ^ md) - (dhost[i] & md));
        }
        if (!c->random_keep) {
            shost[0] &= (uint8_t)~(0x01 * unicast_src);
            dhost[0] &= (uint8_t)~(0x01 * unicast_dst);
        }
    }
    if (newl2len == 14)
        st16(eth + 12, (uint16_t)s->proto);
    if (c->vlan == VLAN_ADD || (c->vlan == VLAN_OFF && s->vlan)) {
        uint8_t *vh = packet + s->vlan_offset; /* {tci, tpid} */
        if (c->vlan == VLAN_ADD) {
            st16(packet + s->l2offset + 12, htons(c->vlan_proto));
            st16(vh + 2, htons((uint16_t)s->proto_vlan_tag));
        }
        if (c->vlan_tag < 65535)
            st16(vh, htons((uint16_t)c->vlan_tag & VIDMASK));
        else if (s->vlan)
            st16(vh, htons(s->vlan_tag));
        if (c->vlan_pri < 255)
            st16(vh, (uint16_t)(ld16(vh) + htons((uint16_t)((uint16_t)c->vlan_pri << 13))));
        else if (s->vlan)
            st16(vh, (uint16_t)(ld16(vh) + htons(s->vlan_pri)));
        if (c->vlan_cfi < 255)
            st16(vh, (uint16_t)(ld16(vh) + htons((uint16_t)((uint16_t)c->vlan_cfi << 12))));
        else if (s->vlan)
            st16(vh, (uint16_t)(ld16(vh) + htons(s->vlan_cfi)));
    } else if (c->vlan == VLAN_DEL && newl2len > 0) {
        st16(eth + 12, htons(s->vlan_proto));
    }
    return pktlen;
}

/* dlt_en10mb_merge_layer3 + multicast MAC update: en10mb.c:797-887 */
static void en10mb_merge_layer3(const ostate_t *s, uint8_t *packet, int pktlen, uint8_t *ip, uint8_t *ip6)
{
    int l2len = en10mb_l2len(packet, pktlen);
    if (l2len == -1 || pktlen < l2len)
        return;
    uint8_t *dhost = packet + s->l2offset;
    if (ip) {
        if ((size_t)pktlen >= 14 + 20 && !s->dst_modified) {
            uint32_t ipd = ld32(ip + 16);
            if (is_multicast_ipv4(ipd)) {
                uint32_t cpu_ip = ntohl(ipd);
                dhost[0] = 0x01;
                dhost[1] = 0x00;
                dhost[2] = 0x5e;
                dhost[3] = (uint8_t)(cpu_ip >> 16) & 0x7f;
                dhost[4] = (uint8_t)(cpu_ip >> 8) & 0xff;
                dhost[5] = (uint8_t)(cpu_ip >> 0) & 0xff;
            }
        }
    } else if (ip6) {
        if ((size_t)pktlen >= 14 + 40 && !s->dst_modified) {
            const uint8_t *a = ip6 + 24;
            if (a[0] == 0xff) {
                dhost[0] = 0x33;
                dhost[1] = 0x33;
                dhost[2] = a[12];
                dhost[3] = a[13];
                dhost[4] = a[14];
                dhost[5] = a[15];
            }
        }
    }
}

/* dlt_user_encode: plugins/dlt_user/user.c:223-268 -- the decoded L2 header
 * (ctx->l2len bytes) replaced by the --user-dlink bytes for the direction */
static int user_encode(const ocfg_t *c, const ostate_t *s, uint8_t *packet, int pktlen, int dir)
{
    if (pktlen == 0)
        return TCPEDIT_ERROR;
    if (s->l2len != c->user_length)
        memmove(packet + c->user_length, packet + s->l2len, (size_t)(pktlen - s->l2len));
    pktlen += c->user_length - s->l2len;
    if (dir == DIR_C2S)
        memcpy(packet, c->user_l2client, (size_t)c->user_length);
    else if (dir == DIR_S2C)
        memcpy(packet, c->user_l2server, (size_t)c->user_length);
    else
        return TCPEDIT_ERROR;
    return pktlen;
}

/* dlt_hdlc_encode: plugins/dlt_hdlc/hdlc.c:223-290 -- a 4-byte Cisco HDLC header
 * {address, control, protocol}.  Without --hdlc-address / --hdlc-control the fields come
 * from `extra->hdlc` (:273, :283): the first int of the context's decoded extra, which no
 * decoder writes as such -- the en10mb decoder's extra begins with its `vlan` flag (1 for
 * a tagged frame, en10mb_types.h:30, en10mb.c:452,466), every other decoder's extra is
 * zeroed and never written there (the HDLC decoder sets only address/control, :212-213).
 * A 0 fails the encode after the memmove (and after the address, when only the control is
 * missing): tcpedit.c:104-108 then writes the record as that left it, a soft error. */
static int hdlc_encode(const ocfg_t *c, const ostate_t *s, uint8_t *packet, int pktlen)
{
    if (pktlen < 4)
        return TCPEDIT_ERROR;
    /* :237-238: after a whole Juniper inner decode the context's decoded extra is the en10mb
       sub-decoder's (dlt_utils.c:262-263), smaller than an hdlc_extra_t: an error before
       anything moves */
    if (c->decoder == DEC_JNPR && s->jnpr_sub)
        return TCPEDIT_ERROR;
    if (s->l2len != 4) /* :241-248 (the l2len < 4 copy writes past pktlen, into the buffer) */
        memmove(packet + 4, packet + s->l2len, (size_t)(pktlen - s->l2len));
    const int newpktlen = pktlen + 4 - s->l2len;
    const int fb = c->decoder == DEC_EN10MB ? s->vlan : 0; /* extra->hdlc */
    if (c->hdlc_address < 65535)
        packet[0] = (uint8_t)c->hdlc_address;
    else if (fb)
        packet[0] = (uint8_t)fb;
    else {
        seterr("Non-HDLC packet requires --hdlc-address");
        return TCPEDIT_ERROR;
    }
    if (c->hdlc_control < 65535)
        packet[1] = (uint8_t)c->hdlc_control;
    else if (fb)
        packet[1] = (uint8_t)fb;
    else {
        seterr("Non-HDLC packet requires --hdlc-control");
        return TCPEDIT_ERROR;
    }
    st16(packet + 2, (uint16_t)s->proto); /* hdlc->protocol = ctx->proto */
    return newpktlen;
}

/* the encoder's L2 length (tcpedit_dlt_l2len on the encoder DLT, tcpedit.c:116):
 * en10mb's parse, user.c:325-342 (the configured length), hdlc.c:355-366 (4) */
static int encoder_l2len(const ocfg_t *c, const uint8_t *packet, int pktlen)
{
    if (c->encoder == ENC_USER)
        return c->user_length;
    if (c->encoder == ENC_HDLC || c->encoder == ENC_PPP) /* pppserial.c:335-343 */
        return pktlen < 4 ? -1 : 4;
    return en10mb_l2len(packet, pktlen);
}

/* ------------------------------------------------------------------------- */
/* fuzzing: src/tcpedit/fuzzing.c:12-297 (state: fuzzing_init's statics)      */
/* ------------------------------------------------------------------------- */
static __thread uint32_t g_fuzz_state, g_fuzz_factor; /* fuzz_seed, fuzz_factor (fuzzing.c:8-20) */
/* test hooks for a sharded run: the draws the last run made, and draws to skip at the
   start of the next runs (a shard's stream starts after the earlier shards' draws) */
static __thread uint64_t g_fuzz_draws, g_fuzz_skip;

/* the encoder's proto function on the edited packet (plugin_proto): en10mb.c:741-762,
   user.c:273-282 (always an error), hdlc.c:299-311 (the protocol field) */
static int encoder_proto(const ocfg_t *c, const uint8_t *packet, int pktlen)
{
    if (c->encoder == ENC_USER)
        return TCPEDIT_ERROR;
    if (c->encoder == ENC_HDLC)
        return pktlen < 4 ? TCPEDIT_ERROR : ld16(packet + 2);
    if (c->encoder == ENC_PPP) /* pppserial.c:257-281 */
        return pktlen < 4 ? TCPEDIT_ERROR : ntohs(ld16(packet + 2)) == 0x0021 ? ETHERTYPE_IP : TCPEDIT_SOFT_ERROR;
    return en10mb_proto(packet, pktlen);
}

#define SGT_MAX_SIZE 16
static int fuzz_get_sgt_size(uint32_t r, uint32_t caplen) /* fuzzing.c:23-35 */
{
    if (caplen == 0)
        return 0;
    if (caplen <= SGT_MAX_SIZE)
        return 1;
    return (int)(1 + (r % (SGT_MAX_SIZE - 1)));
}

static int fuzz_reduce_packet_size(ohdr_t *h, uint32_t new_len) /* fuzzing.c:37-60 */
{
    if (h->len < h->caplen)
        return -1;
    if (new_len > h->caplen)
        return -1;
    if (new_len == h->caplen)
        return 0;
    h->len = new_len;
    h->caplen = h->len;
    return 1;
}

enum { FZ_DROP, FZ_REDUCE, FZ_START_ZERO, FZ_START_RANDOM, FZ_START_FF, FZ_MID_ZERO, FZ_MID_RANDOM, FZ_MID_FF,
       FZ_END_ZERO, FZ_END_RANDOM, FZ_END_FF, FZ_TOTAL }; /* fuzzing.h */

static int oracle_fuzzing(const ocfg_t *c, ohdr_t *h, uint8_t *packet) /* fuzzing.c:62-297 */
{
    int chksum_update_required = 0;
    uint32_t r = tcpr_random(&g_fuzz_state), s;
    g_fuzz_draws++;
    if ((r % g_fuzz_factor) != 0)
        return 0;
    uint8_t *end_ptr = packet + h->caplen, *l4data;
    const int l2len = encoder_l2len(c, packet, (int)h->caplen);
    const uint16_t l2proto = ntohs((uint16_t)encoder_proto(c, packet, (int)h->caplen));
    int l4len;
    uint8_t l4proto;
    if (l2len == -1 || (int)h->caplen < l2len)
        return 0;
    if ((int)h->caplen <= l2len) /* plugin_get_layer3 -> tcpedit_dlt_l3data_copy (dlt_utils.c:196) */
        return 0;
    uint8_t *l3data = packet + l2len;
    switch (l2proto) {
    case ETHERTYPE_IP:
        l4data = get_layer4_v4(packet + l2len, end_ptr);
        if (!l4data)
            return 0;
        l4len = (int)(l4data - packet); /* an offset, as the reference has it */
        l4proto = l3data[9];
        break;
    case ETHERTYPE_IP6:
        l4data = get_layer4_v6(packet + l2len, end_ptr);
        if (!l4data)
            return 0;
        l4len = (int)(l4data - packet);
        l4proto = l3data[6];
        break;
    default:
        l4len = (int)h->caplen - l2len;
        l4data = packet + l2len;
        l4proto = 255; /* IPPROTO_RAW */
    }
    if (l4proto == 6) {
        l4len -= 20;
        l4data += 20;
    } else if (l4proto == 17) {
        l4len -= 8;
        l4data += 8;
    }
    if (l4len <= 1 || l4data > end_ptr)
        return 0;
    r ^= r >> 16;
    s = r % FZ_TOTAL;
    switch (s) {
    case FZ_DROP:
        if (fuzz_reduce_packet_size(h, 0) < 0)
            return 0;
        break;
    case FZ_REDUCE: {
        const uint32_t new_len = (r % (uint32_t)(l4len - 1)) + 1;
        if (fuzz_reduce_packet_size(h, new_len) < 0)
            return 0;
        chksum_update_required = 1;
        break;
    }
    case FZ_START_ZERO: {
        const uint32_t sgt = (uint32_t)fuzz_get_sgt_size(r, (uint32_t)l4len);
        memset(l4data, 0x00, sgt);
        chksum_update_required = 1;
        break;
    }
    case FZ_START_RANDOM: {
        const uint32_t sgt = (uint32_t)fuzz_get_sgt_size(r, (uint32_t)l4len);
        if (!sgt)
            return 0;
        for (uint32_t i = 0; i < sgt; i++)
            l4data[i] = l4data[i] ^ (uint8_t)(r >> 4);
        chksum_update_required = 1;
        break;
    }
    case FZ_START_FF: {
        const uint32_t sgt = (uint32_t)fuzz_get_sgt_size(r, (uint32_t)l4len);
        if (!sgt)
            return 0;
        memset(l4data, 0xff, sgt);
        chksum_update_required = 1;
        break;
    }
    case FZ_MID_ZERO:
    case FZ_MID_FF: {
        if (l4len <= 2)
            return 0;
        const uint32_t offset = ((r >> 16) % (uint32_t)(l4len - 1)) + 1;
        const uint32_t sgt = (uint32_t)fuzz_get_sgt_size(r, (uint32_t)l4len - offset);
        if (!sgt)
            return 0;
        memset(l4data + offset, s == FZ_MID_ZERO ? 0x00 : 0xff, sgt);
        chksum_update_required = 1;
        break;
    }
    case FZ_END_ZERO:
    case FZ_END_FF: {
        const int sgt = fuzz_get_sgt_size(r, (uint32_t)l4len);
        if (!sgt || sgt > l4len)
            return 0;
        memset(l4data + l4len - sgt, s == FZ_END_ZERO ? 0x00 : 0xff, (size_t)sgt);
        chksum_update_required = 1;
        break;
    }
    case FZ_END_RANDOM: {
        const int sgt = fuzz_get_sgt_size(r, (uint32_t)l4len);
        if (!sgt || sgt > l4len)
            return 0;
        for (int i = l4len - sgt; i < l4len; i++)
            l4data[i] = l4data[i] ^ (uint8_t)(r >> 4);
        chksum_update_required = 1;
        break;
    }
    case FZ_MID_RANDOM: {
        const uint32_t offset = ((r >> 16) % (uint32_t)(l4len - 1)) + 1;
        const int sgt = fuzz_get_sgt_size(r, (uint32_t)l4len - offset);
        if (!sgt || sgt > l4len)
            return 0;
        for (uint32_t i = offset; i < offset + (uint32_t)sgt; i++)
            l4data[i] = l4data[i] ^ (uint8_t)(r >> 4);
        chksum_update_required = 1;
        break;
    }
    }
    return chksum_update_required;
}

/* ------------------------------------------------------------------------- */
/* tcpedit_packet: src/tcpedit/tcpedit.c:46-366                              */
/* ------------------------------------------------------------------------- */
static int oracle_tcpedit_packet(const ocfg_t *c, ostate_t *s, ohdr_t *h, uint8_t *packet, int direction, int *warned)
{
    uint8_t *ip = NULL, *ip6 = NULL;
    int l2len, l2proto, retval = 0, pktlen, lendiff, needtorecalc = 0;
    *warned = 0;

    if (c->efcs && h->len > 4) { /* :78-84 */
        if (h->caplen == h->len)
            h->caplen -= 4;
        h->len -= 4;
    }
    int fuzz_once = c->fuzz_seed != 0; /* :48 */
again: /* :89 -- a fuzzed packet goes through L2 and the per-family edits once more */
    ip = ip6 = NULL;
    retval = 0;
    if ((l2proto = decoder_proto(c, packet, (int)h->caplen)) < 0) /* :96 */
        return TCPEDIT_SOFT_ERROR;

    /* tcpedit_dlt_process: dlt_plugins.c:210-238 */
    if (direction == DIR_NOSEND) {
        pktlen = (int)h->caplen;
    } else {
        int rc = decoder_decode(c, s, packet, (int)h->caplen);
        if (rc == TCPEDIT_ERROR || rc == TCPEDIT_SOFT_ERROR) /* (a TCPEDIT_WARN goes on to encode) */
            return TCPEDIT_SOFT_ERROR;
        if (c->encoder == ENC_USER)
            pktlen = user_encode(c, s, packet, (int)h->caplen, direction);
        else if (c->encoder == ENC_HDLC)
            pktlen = hdlc_encode(c, s, packet, (int)h->caplen);
        else if (c->encoder == ENC_NOENC) /* linuxsll.c:201-208 and the like */
            pktlen = TCPEDIT_ERROR;
        else if (c->encoder == ENC_PPP) /* pppserial.c:239-251 */
            pktlen = h->caplen < 4 ? TCPEDIT_ERROR : (int)h->caplen;
        else
            pktlen = en10mb_encode(c, s, packet, (int)h->caplen, direction);
        if (pktlen < 0)
            return TCPEDIT_SOFT_ERROR;
    }
    lendiff = pktlen - (int)h->caplen; /* :111-113 */
    h->caplen += lendiff;
    h->len += lendiff;

    l2len = encoder_l2len(c, packet, (int)h->caplen); /* :116 */
    if (l2len == -1)
        return TCPEDIT_SOFT_ERROR;

    if (l2proto == htons(ETHERTYPE_IP)) { /* :123-148 */
        if (h->caplen < (uint32_t)l2len + 20)
            return TCPEDIT_SOFT_ERROR;
        int l2 = encoder_l2len(c, packet, (int)h->caplen); /* the encoder's get_layer3 (en10mb.c:768-779, user.c:284-298, hdlc.c:313-330) */
        if (l2 == -1 || (int)h->caplen < l2 || (int)h->caplen <= l2)
            return TCPEDIT_SOFT_ERROR;
        ip = packet + l2;
        if (!get_layer4_v4(ip, ip + h->caplen - l2len))
            return TCPEDIT_SOFT_ERROR;
    } else if (l2proto == htons(ETHERTYPE_IP6)) { /* :149-173 */
        if (h->caplen < (uint32_t)l2len + 40)
            return TCPEDIT_SOFT_ERROR;
        int l2 = encoder_l2len(c, packet, (int)h->caplen);
        if (l2 == -1 || (int)h->caplen < l2 || (int)h->caplen <= l2)
            return TCPEDIT_SOFT_ERROR;
        ip6 = packet + l2;
        if (!get_layer4_v6(ip6, ip6 + h->caplen - l2len))
            return TCPEDIT_SOFT_ERROR;
    }

    int l3len = (int)h->caplen - l2len;
    if (ip != NULL) { /* :182-206 */
        if (c->tos > -1) {
            uint16_t oldval = ld16(ip);
            uint16_t newval = htons((uint16_t)((ntohs(oldval) & 0xff00) | (c->tos & 0xff)));
            st16(ip, newval);
            csum_replace2(ip + 10, oldval, newval);
        }
        needtorecalc += rewrite_ipv4_ttl(c, ip);
        if (c->n_portmap > 0) {
            retval = rewrite_ipv4_ports(c, ip, l3len);
            needtorecalc += retval;
        }
        if (c->tcp_sequence_enable)
            rewrite_ipv4_tcp_sequence(c, ip, l3len);
    } else if (ip6 != NULL) { /* :209-248 */
        needtorecalc += rewrite_ipv6_hlim(c, ip6);
        if (c->tclass > -1) {
            uint32_t ipflags = ntohl(ld32(ip6)) & 0xf00fffff;
            ipflags += (uint32_t)c->tclass << 20;
            st32(ip6, htonl(ipflags));
        }
        if (c->flowlabel > -1) {
            uint32_t ipflags = ntohl(ld32(ip6)) & 0xfff00000;
            ipflags += (uint32_t)c->flowlabel;
            st32(ip6, htonl(ipflags));
        }
        if (c->n_portmap > 0) {
            retval = rewrite_ipv6_ports(c, ip6, l3len);
            needtorecalc += retval;
        }
        if (c->tcp_sequence_enable)
            rewrite_ipv6_tcp_sequence(c, ip6, l3len);
    }

    if (fuzz_once) { /* :250-258 */
        fuzz_once = 0;
        retval = oracle_fuzzing(c, h, packet);
        needtorecalc += retval;
        goto again;
    }

    if (c->fixlen || c->mtu_truncate) { /* :261-265 */
        if ((retval = untrunc_packet(c, h, packet, ip, ip6)) < 0)
            return TCPEDIT_ERROR;
        needtorecalc += retval;
    }

    l3len = (int)h->caplen - l2len;
    if (c->rewrite_ip) { /* :268-290 */
        if (ip != NULL) {
            retval = rewrite_ipv4l3(c, ip, direction, l3len);
            needtorecalc += retval;
        } else if (ip6 != NULL) {
            retval = rewrite_ipv6l3(c, ip6, direction, l3len);
            needtorecalc += retval;
        } else if (l2proto == htons(ETHERTYPE_ARP)) {
            rewrite_iparp(c, packet + l2len, direction);
        }
    }

    if (c->seed) { /* :293-317 */
        if (ip != NULL) {
            if ((retval = randomize_ipv4(c, h, ip, l3len)) < 0)
                return TCPEDIT_ERROR;
            needtorecalc += retval;
        } else if (ip6 != NULL) {
            if ((retval = randomize_ipv6(c, h, ip6, l3len)) < 0)
                return TCPEDIT_ERROR;
            needtorecalc += retval;
        } else if (l2proto == htons(ETHERTYPE_ARP)) {
            if (randomize_iparp(c, h, packet, l3len) < 0)
                return TCPEDIT_ERROR;
        }
    }

    if (c->fixhdrlen) { /* :321-335 */
        int changed = 0;
        if (ip != NULL)
            changed = fix_ipv4_length(h, ip, (size_t)l2len);
        else if (ip6 != NULL)
            changed |= fix_ipv6_length(h, ip6, (size_t)l2len);
        if (changed > 0)
            needtorecalc |= changed;
    }

    if (c->fixcsum || needtorecalc > 0) { /* :338-354 */
        if (ip != NULL)
            retval = fix_ipv4_checksums(h, ip, (size_t)l2len);
        else if (ip6 != NULL)
            retval = fix_ipv6_checksums(h, ip6, (size_t)l2len);
        else
            retval = TCPEDIT_OK;
        if (retval < 0)
            return TCPEDIT_ERROR;
        else if (retval == TCPEDIT_WARN)
            *warned = 1;
    }

    if (c->encoder == ENC_EN10MB) /* :356-361; user/hdlc merge in place (dlt_utils.c:189-221) */
        en10mb_merge_layer3(s, packet, (int)h->caplen, ip, ip6);
    return retval;
}

/* ------------------------------------------------------------------------- */
/* option parsing: parse_args.c:34-254, cidr.c:130-418, portmap.c:55-218,    */
/* mac.c:33-104, en10mb.c:226-396                                            */
/* ------------------------------------------------------------------------- */
enum {
    O_PORTMAP, O_SEED, O_PNAT, O_SRCIPMAP, O_DSTIPMAP, O_ENDPOINTS, O_TCP_SEQUENCE, O_SKIPBROADCAST, O_FIXCSUM,
    O_FIXHDRLEN, O_MTU, O_MTU_TRUNC, O_EFCS, O_TTL, O_TOS, O_TCLASS, O_FLOWLABEL, O_FIXLEN, O_FUZZ_SEED,
    O_FUZZ_FACTOR, O_DLT, O_SKIPL2BROADCAST, O_ENET_DMAC, O_ENET_SMAC, O_ENET_SUBSMAC, O_ENET_MAC_SEED,
    O_ENET_MAC_SEED_KEEP_BYTES, O_ENET_VLAN, O_ENET_VLAN_TAG, O_ENET_VLAN_CFI, O_ENET_VLAN_PRI, O_ENET_VLAN_PROTO,
    O_SKIP_SOFT_ERRORS, O_CACHEFILE, O_INFILE, O_OUTFILE, O_USER_DLT, O_USER_DLINK, O_HDLC_CONTROL,
    O_HDLC_ADDRESS, O__N
};
static const struct {
    const char *name;
    char shortopt;
    int has_arg;
    int stacked;
} g_opts[O__N] = {
    [O_PORTMAP] = {"portmap", 'r', 1, 1},
    [O_SEED] = {"seed", 's', 1, 0},
    [O_PNAT] = {"pnat", 'N', 1, 1},
    [O_SRCIPMAP] = {"srcipmap", 'S', 1, 0},
    [O_DSTIPMAP] = {"dstipmap", 'D', 1, 0},
    [O_ENDPOINTS] = {"endpoints", 'e', 1, 0},
    [O_TCP_SEQUENCE] = {"tcp-sequence", 0, 1, 0},
    [O_SKIPBROADCAST] = {"skipbroadcast", 'b', 0, 0},
    [O_FIXCSUM] = {"fixcsum", 'C', 0, 0},
    [O_FIXHDRLEN] = {"fixhdrlen", 0, 0, 0},
    [O_MTU] = {"mtu", 'm', 1, 0},
    [O_MTU_TRUNC] = {"mtu-trunc", 0, 0, 0},
    [O_EFCS] = {"efcs", 'E', 0, 0},
    [O_TTL] = {"ttl", 0, 1, 0},
    [O_TOS] = {"tos", 0, 1, 0},
    [O_TCLASS] = {"tclass", 0, 1, 0},
    [O_FLOWLABEL] = {"flowlabel", 0, 1, 0},
    [O_FIXLEN] = {"fixlen", 'F', 1, 0},
    [O_FUZZ_SEED] = {"fuzz-seed", 0, 1, 0},
    [O_FUZZ_FACTOR] = {"fuzz-factor", 0, 1, 0},
    [O_DLT] = {"dlt", 0, 1, 0},
    [O_SKIPL2BROADCAST] = {"skipl2broadcast", 0, 0, 0},
    [O_ENET_DMAC] = {"enet-dmac", 0, 1, 0},
    [O_ENET_SMAC] = {"enet-smac", 0, 1, 0},
    [O_ENET_SUBSMAC] = {"enet-subsmac", 0, 1, 1},
    [O_ENET_MAC_SEED] = {"enet-mac-seed", 0, 1, 0},
    [O_ENET_MAC_SEED_KEEP_BYTES] = {"enet-mac-seed-keep-bytes", 0, 1, 0},
    [O_ENET_VLAN] = {"enet-vlan", 0, 1, 0},
    [O_ENET_VLAN_TAG] = {"enet-vlan-tag", 0, 1, 0},
    [O_ENET_VLAN_CFI] = {"enet-vlan-cfi", 0, 1, 0},
    [O_ENET_VLAN_PRI] = {"enet-vlan-pri", 0, 1, 0},
    [O_ENET_VLAN_PROTO] = {"enet-vlan-proto", 0, 1, 0},
    [O_SKIP_SOFT_ERRORS] = {"skip-soft-errors", 0, 0, 0},
    [O_CACHEFILE] = {"cachefile", 'c', 1, 0},
    [O_INFILE] = {"infile", 'i', 1, 0},
    [O_OUTFILE] = {"outfile", 'o', 1, 0},
    [O_USER_DLT] = {"user-dlt", 0, 1, 0},     /* user_opts.def */
    [O_USER_DLINK] = {"user-dlink", 0, 1, 1},
    [O_HDLC_CONTROL] = {"hdlc-control", 0, 1, 0}, /* hdlc_opts.def */
    [O_HDLC_ADDRESS] = {"hdlc-address", 0, 1, 0},
};

typedef struct {
    int have[O__N];
    const char *arg[O__N];
    const char *stack[O__N][64];
    int nstack[O__N];
} oopts_t;

static int parse_argv(oopts_t *o, int argc, const char **argv)
{
    memset(o, 0, sizeof(*o));
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i];
        int idx = -1;
        const char *val = NULL;
        if (a[0] == '-' && a[1] == '-') {
            const char *eq = strchr(a + 2, '=');
            size_t n = eq ? (size_t)(eq - (a + 2)) : strlen(a + 2);
            for (int k = 0; k < O__N; k++)
                if (strlen(g_opts[k].name) == n && strncmp(g_opts[k].name, a + 2, n) == 0)
                    idx = k;
            if (idx < 0) {
                seterr("unknown option %s", a);
                return -1;
            }
            if (g_opts[idx].has_arg) {
                if (eq)
                    val = eq + 1;
                else if (i + 1 < argc)
                    val = argv[++i];
                else {
                    seterr("option %s needs an argument", a);
                    return -1;
                }
            }
        } else if (a[0] == '-' && a[1] && !a[2]) {
            for (int k = 0; k < O__N; k++)
                if (g_opts[k].shortopt == a[1])
                    idx = k;
            if (idx < 0) {
                seterr("unknown option %s", a);
                return -1;
            }
            if (g_opts[idx].has_arg) {
                if (i + 1 >= argc) {
                    seterr("option %s needs an argument", a);
                    return -1;
                }
                val = argv[++i];
            }
        } else {
            seterr("unexpected argument %s", a);
            return -1;
        }
        o->have[idx] = 1;
        o->arg[idx] = val;
        if (g_opts[idx].stacked && o->nstack[idx] < 64)
            o->stack[idx][o->nstack[idx]++] = val;
    }
    return 0;
}

static long opt_num(const oopts_t *o, int idx) { return strtol(o->arg[idx], NULL, 0); }

/* read_hexstring: src/common/utils.c:331-380 -- comma-separated hex bytes (strtol base
 * 16, so "0x0f" and "f" alike); -1 where the reference errx()s on a byte > 0xff */
static int read_hexstring(const char *l2string, uint8_t *hex, int hexlen)
{
    char buf[4096];
    int numbytes = 0;
    snprintf(buf, sizeof(buf), "%s", l2string);
    memset(hex, 0, (size_t)hexlen);
    char *save = NULL, *tok = strtok_r(buf, ",", &save);
    if (!tok)
        return -1;
    for (; tok; tok = strtok_r(NULL, ",", &save)) {
        if (numbytes + 1 > hexlen)
            break; /* "Hex buffer too small for data- skipping data" */
        const unsigned long v = strtoul(tok, NULL, 16);
        if (v > 0xff)
            return -1;
        hex[numbytes++] = (uint8_t)v;
    }
    return numbytes;
}

/* cidr2cidr: cidr.c:130-221 */
static int cidr2cidr(char *cidr, ocidr_t *out)
{
    unsigned int octets[4];
    int count;
    memset(out, 0, sizeof(*out));
    out->masklen = 99;
    for (char *p = cidr; *p; ++p) {
        if (*p == '#')
            *p = ':';
        else if (*p == ']') {
            *p = 0;
            break;
        }
    }
    count = sscanf(cidr, "%u.%u.%u.%u/%d", &octets[0], &octets[1], &octets[2], &octets[3], &out->masklen);
    if (count == 4) {
        out->masklen = 32;
        out->family = 4;
    } else if (count == 5) {
        out->family = 4;
    } else {
        char *p = strstr(cidr, "/");
        if (p) {
            *p = 0;
            ++p;
            sscanf(p, "%d", &out->masklen);
        } else {
            out->masklen = 128;
        }
        if (out->masklen < 0 || out->masklen > 128)
            return 0;
        if (*cidr == '[')
            cidr++;
        if (inet_pton(AF_INET6, cidr, out->network6) > 0)
            out->family = 6;
        else
            return 0;
    }
    if (out->family == 4) {
        if (out->masklen > 32)
            return 0;
        char networkip[16] = {0}, tempoctet[4];
        for (count = 0; count < 4; count++) {
            if (octets[count] > 255)
                return 0;
            snprintf(tempoctet, sizeof(octets[count]), "%u", octets[count]);
            strcat(networkip, tempoctet);
            if (count < 3)
                strcat(networkip, ".");
        }
        struct in_addr ia;
        inet_aton(networkip, &ia);
        out->network = ia.s_addr;
    }
    return 1;
}

static void mask_cidr6(char **cidrin, const char *delim) /* cidr.c:223-236 */
{
    if (**cidrin == '[' && *delim == ':') {
        ++*cidrin;
        for (char *p = *cidrin; *p && *p != ']'; ++p)
            if (*p == ':')
                *p = '#';
    }
}

/* parse_cidr with delim ":" producing a list (cidr.c:244-279) */
static int parse_cidr_list(ocidr_t *outv, int maxn, int *n, char *cidrin)
{
    char *token = NULL, *network;
    *n = 0;
    if (!cidrin)
        return 0;
    mask_cidr6(&cidrin, ":");
    network = strtok_r(cidrin, ":", &token);
    if (network == NULL)
        return 0;
    if (!cidr2cidr(network, &outv[(*n)++]))
        return -1;
    for (;;) {
        if (token)
            mask_cidr6(&token, ":");
        network = strtok_r(NULL, ":", &token);
        if (network == NULL)
            break;
        if (*n >= maxn)
            return -1;
        if (!cidr2cidr(network, &outv[(*n)++]))
            return -1;
    }
    return 1;
}

/* parse_cidr_map: cidr.c:371-418 (appends pairs) */
static int parse_cidr_map(ocidrmap_t **maps, int *nmaps, const char *optarg)
{
    char *string = strdup(optarg), *token = NULL, *map;
    int res = 0;
    ocidr_t tmp[8];
    int n;
    *maps = NULL;
    *nmaps = 0;
    map = strtok_r(string, ",", &token);
    for (int first = 1;; first = 0) {
        if (!first) {
            map = strtok_r(NULL, ",", &token);
            if (map == NULL)
                break;
        }
        int rc = parse_cidr_list(tmp, 8, &n, map);
        if (rc < 0) {
            seterr("Unable to parse as a valid CIDR");
            free(string);
            return -2; /* the reference errx()s inside cidr2cidr (cidr.c:221) */
        }
        if (rc == 0 || n < 2)
            goto done;
        *maps = realloc(*maps, sizeof(ocidrmap_t) * (*nmaps + 1));
        (*maps)[*nmaps].from = tmp[0];
        (*maps)[*nmaps].to = tmp[1];
        (*nmaps)++;
    }
    res = 1;
done:
    free(string);
    return res;
}

/* parse_endpoints: cidr.c:290-362 */
static int parse_endpoints(ocfg_t *c, const char *optarg)
{
    char newmap[128];
    char *string = strdup(optarg), *token = NULL, *map;
    int res = 0;
    if (*string == '[') {
        char *p = strstr(string, "]:[");
        if (!p)
            goto done;
        *p = 0;
        snprintf(newmap, sizeof(newmap), "[::/0]:%s]", string);
        if (parse_cidr_map(&c->cidrmap1, &c->n_cidrmap1, newmap) != 1)
            goto done;
        snprintf(newmap, sizeof(newmap), "[::/0]:%s", p + 2);
        if (parse_cidr_map(&c->cidrmap2, &c->n_cidrmap2, newmap) != 1)
            goto done;
    } else {
        map = strtok_r(string, ":", &token);
        if (map == NULL)
            goto done;
        snprintf(newmap, sizeof(newmap), "0.0.0.0/0:%s", map);
        if (parse_cidr_map(&c->cidrmap1, &c->n_cidrmap1, newmap) != 1)
            goto done;
        map = strtok_r(NULL, ":", &token);
        if (map == NULL)
            goto done;
        snprintf(newmap, sizeof(newmap), "0.0.0.0/0:%s", map);
        if (parse_cidr_map(&c->cidrmap2, &c->n_cidrmap2, newmap) != 1)
            goto done;
    }
    res = 1;
done:
    free(string);
    return res;
}

static void portmap_push(ocfg_t *c, long from, long to)
{
    c->portmap = realloc(c->portmap, sizeof(oport_t) * (c->n_portmap + 1));
    c->portmap[c->n_portmap].from = from;
    c->portmap[c->n_portmap].to = to;
    c->n_portmap++;
}

/* ports2PORT: portmap.c:55-170 -- appends the chain to c->portmap; returns 0 on failure */
static int ports2PORT(ocfg_t *c, char *ports)
{
    char *token = NULL, *token2 = NULL, *badchar, *from_s, *to_s;
    long from_l, to_l;
    from_s = strtok_r(ports, ":", &token);
    to_s = strtok_r(NULL, ":", &token);
    if (strtok_r(NULL, ":", &token) != NULL)
        return 0;
    if (from_s == NULL || to_s == NULL)
        return 0;
    if (strchr(from_s, '-') && strchr(from_s, '+'))
        return 0;
    to_l = strtol(to_s, &badchar, 10);
    if (strlen(badchar) != 0)
        return 0;
    if (to_l > 65535 || to_l < 0)
        return 0;
    if (strchr(from_s, '-')) {
        char *from_begin = strtok_r(from_s, "-", &token2);
        char *from_end = strtok_r(NULL, "-", &token2);
        long from_b = strtol(from_begin, &badchar, 10);
        if (!from_begin || !from_end || strlen(badchar) != 0)
            return 0;
        long from_e = strtol(from_end, &badchar, 10);
        if (from_b > 65535 || from_b < 0 || from_e > 65535 || from_e < 0)
            return 0;
        for (long i = from_b; i <= from_e; i++)
            portmap_push(c, htons((uint16_t)i), htons((uint16_t)to_l));
        portmap_push(c, 0, 0); /* the trailing zeroed node the range loop leaves (portmap.c:117-124) */
    } else if (strchr(from_s, '+')) {
        char *from_begin = strtok_r(from_s, "+", &token2);
        from_l = strtol(from_begin, &badchar, 10);
        if (strlen(badchar) != 0)
            return 0;
        int start = c->n_portmap;
        portmap_push(c, htons((uint16_t)from_l), htons((uint16_t)to_l));
        while ((from_begin = strtok_r(NULL, "+", &token2)) != NULL) {
            from_l = strtol(from_begin, &badchar, 10);
            if (strlen(badchar) != 0 || from_l > 65535 || from_l < 0) {
                c->n_portmap = start;
                return 0;
            }
            portmap_push(c, htons((uint16_t)from_l), htons((uint16_t)to_l));
        }
    } else {
        from_l = strtol(from_s, &badchar, 10);
        if (strlen(badchar) != 0 || from_l > 65535 || from_l < 0)
            return 0;
        portmap_push(c, htons((uint16_t)from_l), htons((uint16_t)to_l));
    }
    return 1;
}

/* parse_portmap: portmap.c:179-218 (a failing later record is silently dropped) */
static int parse_portmap(ocfg_t *c, const char *ourstr)
{
    char *copy = strdup(ourstr), *token = NULL;
    char *substr = strtok_r(copy, ",", &token);
    if (substr == NULL || !ports2PORT(c, substr)) {
        free(copy);
        return 0;
    }
    while ((substr = strtok_r(NULL, ",", &token)) != NULL)
        ports2PORT(c, substr);
    free(copy);
    return 1;
}

/* mac2hex / dualmac2hex: mac.c:33-104 */
static void mac2hex(const char *mac, uint8_t *dst, int len)
{
    char *pp;
    if (len < 6)
        return;
    while (isspace((unsigned char)*mac))
        mac++;
    for (int i = 0; i < 6; i++) {
        long l = strtol(mac, &pp, 16);
        if (pp == mac || l > 0xFF || l < 0)
            return;
        if (!(*pp == ':' || (i == 5 && (isspace((unsigned char)*pp) || *pp == '\0'))))
            return;
        dst[i] = (uint8_t)l;
        mac = pp + 1;
    }
}
static int dualmac2hex(const char *dualmac, uint8_t *first, uint8_t *second, int len)
{
    char *tok = NULL, *temp, *string = strdup(dualmac);
    int ret = 0;
    if (len <= 1)
        goto done;
    temp = strtok_r(string, ",", &tok);
    if (temp && strlen(temp)) {
        mac2hex(temp, first, len);
        ret = 1;
    }
    temp = strtok_r(NULL, ",", &tok);
    if (temp != NULL && strlen(temp)) {
        mac2hex(temp, second, len);
        ret += 2;
    }
done:
    free(string);
    return ret;
}

/* tcpedit_post_args (parse_args.c:34-254) + dlt_en10mb_parse_opts (en10mb.c:226-396) */
static int oracle_post_args(ocfg_t *c, const oopts_t *o)
{
    uint32_t seed = 1, rand_num = 0;
    const int decoder = c->decoder, in_dlt = c->in_dlt; /* set from the input DLT */
    memset(c, 0, sizeof(*c));
    c->decoder = decoder;
    c->in_dlt = in_dlt;
    c->mtu = DEFAULT_MTU; /* tcpedit.c:382-390 */
    c->tos = -1;
    c->tclass = -1;
    c->flowlabel = -1;
    c->vlan_tag = 65535; /* en10mb.c:117-122 */
    c->vlan_pri = 255;
    c->vlan_cfi = 255;
    c->vlan_proto = ETHERTYPE_VLAN;

    if (o->have[O_PNAT]) {
        c->rewrite_ip = true;
        for (int k = 0; k < o->nstack[O_PNAT] && k < 2; k++) {
            int rc = k == 0 ? parse_cidr_map(&c->cidrmap1, &c->n_cidrmap1, o->stack[O_PNAT][k])
                            : parse_cidr_map(&c->cidrmap2, &c->n_cidrmap2, o->stack[O_PNAT][k]);
            if (rc != 1) {
                seterr("Unable to parse %s --pnat=%s", k == 0 ? "first" : "second", o->stack[O_PNAT][k]);
                return -1;
            }
        }
    }
    if (o->have[O_SRCIPMAP]) {
        c->rewrite_ip = true;
        if (parse_cidr_map(&c->srcipmap, &c->n_srcipmap, o->arg[O_SRCIPMAP]) != 1) {
            seterr("Unable to parse --srcipmap=%s", o->arg[O_SRCIPMAP]);
            return -1;
        }
    }
    if (o->have[O_DSTIPMAP]) {
        c->rewrite_ip = true;
        if (parse_cidr_map(&c->dstipmap, &c->n_dstipmap, o->arg[O_DSTIPMAP]) != 1) {
            seterr("Unable to parse --dstipmap=%s", o->arg[O_DSTIPMAP]);
            return -1;
        }
    }
    if (c->n_cidrmap1 && !c->n_cidrmap2) {
        c->cidrmap2 = c->cidrmap1;
        c->n_cidrmap2 = c->n_cidrmap1;
    }
    if (o->have[O_FIXCSUM])
        c->fixcsum = true;
    if (o->have[O_FIXHDRLEN])
        c->fixhdrlen = true;
    if (o->have[O_EFCS])
        c->efcs = true;
    if (o->have[O_TTL]) {
        const char *a = o->arg[O_TTL];
        if (strchr(a, '+'))
            c->ttl_mode = TTL_ADD;
        else if (strchr(a, '-'))
            c->ttl_mode = TTL_SUB;
        else
            c->ttl_mode = TTL_SET;
        long ttl = strtol(a, NULL, 10);
        if (ttl < 0)
            ttl *= -1;
        if (ttl > 255) {
            seterr("Invalid --ttl value (must be 0-255): %ld", ttl);
            return -1;
        }
        c->ttl_value = (uint8_t)ttl;
    }
    if (o->have[O_TOS])
        c->tos = (int)opt_num(o, O_TOS);
    if (o->have[O_TCLASS])
        c->tclass = (int)opt_num(o, O_TCLASS);
    if (o->have[O_FLOWLABEL])
        c->flowlabel = (int)opt_num(o, O_FLOWLABEL);
    if (o->have[O_MTU])
        c->mtu = (int)opt_num(o, O_MTU);
    if (o->have[O_MTU_TRUNC])
        c->mtu_truncate = true;
    if (o->have[O_SKIPBROADCAST])
        c->skip_broadcast = true;
    if (o->have[O_FIXLEN]) {
        const char *a = o->arg[O_FIXLEN];
        if (!strcmp(a, "pad"))
            c->fixlen = FIXLEN_PAD;
        else if (!strcmp(a, "trunc"))
            c->fixlen = FIXLEN_TRUNC;
        else if (!strcmp(a, "del"))
            c->fixlen = FIXLEN_DEL;
        else {
            seterr("Invalid --fixlen=%s", a);
            return -1;
        }
    }
    if (o->have[O_TCP_SEQUENCE]) {
        c->tcp_sequence_enable = 1;
        seed = (uint32_t)opt_num(o, O_TCP_SEQUENCE);
        for (int i = 0; i < 5; ++i)
            rand_num = tcpr_random(&seed);
        c->tcp_sequence_adjust = rand_num;
    }
    if (o->have[O_PORTMAP]) {
        for (int k = 0; k < o->nstack[O_PORTMAP]; k++) {
            if (!parse_portmap(c, o->stack[O_PORTMAP][k])) {
                seterr("Unable to parse --portmap=%s", o->stack[O_PORTMAP][k]);
                return -1;
            }
        }
    }
    if (o->have[O_SEED] && o->have[O_FUZZ_SEED]) { /* seed: flags-cant = fuzz-seed (tcpedit_opts.def:46-48) */
        seterr("--seed and --fuzz-seed are mutually exclusive");
        return -1;
    }
    if (o->have[O_FUZZ_FACTOR] && !o->have[O_FUZZ_SEED]) { /* fuzz-factor: flags-must = fuzz-seed (:324-326) */
        seterr("--fuzz-factor requires --fuzz-seed");
        return -1;
    }
    if (o->have[O_SEED]) {
        c->rewrite_ip = true;
        seed = (uint32_t)opt_num(o, O_SEED);
    } else if (o->have[O_FUZZ_SEED]) {
        seed = (uint32_t)opt_num(o, O_FUZZ_SEED);
    }
    for (int i = 0; i < 5; ++i)
        rand_num = tcpr_random(&seed);
    if (o->have[O_SEED])
        c->seed = seed;
    if (o->have[O_FUZZ_SEED]) {
        c->fuzz_seed = seed;
        c->fuzz_factor = o->have[O_FUZZ_FACTOR] ? (uint32_t)opt_num(o, O_FUZZ_FACTOR) : 8;
        if (c->fuzz_factor < 1) {
            seterr("--fuzz-factor must be >= 1");
            return -1;
        }
    }
    if (o->have[O_ENDPOINTS]) {
        c->rewrite_ip = true;
        if (!parse_endpoints(c, o->arg[O_ENDPOINTS])) {
            seterr("Unable to parse --endpoints=%s", o->arg[O_ENDPOINTS]);
            return -1;
        }
    }
    /* tcpedit_dlt_post_args: dlt_plugins.c:168-204 -- the encoder by name */
    /* the decoder's own plugin unless --dlt names another (plugin->name: en10mb.c:61,
       linuxsll.c:63, linuxsll2.c:66, raw.c:63, null.c:80, loop.c:69, pppserial.c:71,
       hdlc.c:62, user.c:62) */
    {
        static const struct {
            const char *name;
            int enc, dlt;
        } plugins[] = {{"enet", ENC_EN10MB, 1},      {"user", ENC_USER, 147},    {"hdlc", ENC_HDLC, 104},
                       {"linuxsll", ENC_NOENC, 113}, {"linuxsll2", ENC_NOENC, 276}, {"raw", ENC_NOENC, 12},
                       {"null", ENC_NOENC, 0},       {"loop", ENC_NOENC, 108},   {"pppserial", ENC_PPP, 50},
                       {"jnpr_eth", ENC_NOENC, 178}, {"ieee80211", ENC_NOENC, 105}, {"radiotap", ENC_NOENC, 127}};
        static const int dec_enc[] = {[DEC_EN10MB] = ENC_EN10MB, [DEC_SLL] = ENC_NOENC, [DEC_SLL2] = ENC_NOENC,
                                      [DEC_RAW] = ENC_NOENC,     [DEC_NULL] = ENC_NOENC, [DEC_PPP] = ENC_PPP,
                                      [DEC_CHDLC] = ENC_HDLC,    [DEC_JNPR] = ENC_NOENC, [DEC_80211] = ENC_NOENC,
                                      [DEC_RADIOTAP] = ENC_NOENC};
        c->encoder = dec_enc[c->decoder];
        c->out_linktype = c->in_dlt;
        if (o->have[O_DLT]) {
            int k = 0, n = (int)(sizeof(plugins) / sizeof(plugins[0]));
            while (k < n && strcmp(plugins[k].name, o->arg[O_DLT]) != 0)
                k++;
            if (k == n) {
                seterr("No output DLT plugin available for: %s", o->arg[O_DLT]);
                return -1;
            }
            c->encoder = plugins[k].enc;
            c->out_linktype = plugins[k].dlt;
        }
    }
    c->user_length = -1;
    c->hdlc_address = c->hdlc_control = 65535;
    /* dlt_user_parse_opts: user.c:158-205 (--user-dlt, else the decoder's DLT) */
    if (o->have[O_USER_DLT])
        c->user_dlt_set = 1, c->user_dlt = (int)opt_num(o, O_USER_DLT);
    if (c->encoder == ENC_USER)
        c->out_linktype = c->user_dlt_set ? c->user_dlt : c->in_dlt;
    if (o->have[O_USER_DLINK]) {
        for (int k = 0; k < o->nstack[O_USER_DLINK]; k++) {
            uint8_t *dst = k == 0 ? c->user_l2server : c->user_l2client;
            const int n = read_hexstring(o->stack[O_USER_DLINK][k], dst, 255);
            if (n < 0) {
                seterr("Invalid hex string: %s", o->stack[O_USER_DLINK][k]);
                return -1;
            }
            if (k == 0) {
                c->user_length = n;
                memcpy(c->user_l2client, c->user_l2server, (size_t)n);
            } else if (n != c->user_length) {
                seterr("both --dlink's must contain the same number of bytes");
                return -1;
            }
        }
    }
    if (c->encoder == ENC_USER && c->user_length < 0) {
        seterr("--dlt=user requires --user-dlink");
        return -1;
    }
    /* dlt_hdlc_parse_opts: hdlc.c:156-180 */
    if (o->have[O_HDLC_CONTROL])
        c->hdlc_control = (uint16_t)opt_num(o, O_HDLC_CONTROL);
    if (o->have[O_HDLC_ADDRESS])
        c->hdlc_address = (uint16_t)opt_num(o, O_HDLC_ADDRESS);
    if (o->have[O_SKIPL2BROADCAST])
        c->l2_skip_broadcast = true;
    /* dlt_en10mb_parse_opts: en10mb.c:226-396 */
    if (o->have[O_ENET_SUBSMAC]) {
        for (int k = 0; k < o->nstack[O_ENET_SUBSMAC]; k++) {
            const char *input = o->stack[O_ENET_SUBSMAC][k];
            size_t input_len = strlen(input);
            size_t possible = (input_len / 36) + 1; /* SUBSMAC_ENTRY_LEN + 1 (en10mb.h:27) */
            for (size_t e = 0; e < possible; e++) {
                size_t off = e + e * 35;
                if (input_len - off < 35) {
                    seterr("Unable to parse --enet-subsmac=%s", input);
                    return -1;
                }
                uint8_t t[6] = {0}, r[6] = {0};
                if (dualmac2hex(input + off, t, r, 35) != 3) {
                    seterr("Unable to parse --enet-subsmac=%s", input);
                    return -1;
                }
                c->subs = realloc(c->subs, sizeof(*c->subs) * (c->n_subs + 1));
                memcpy(c->subs[c->n_subs][0], t, 6);
                memcpy(c->subs[c->n_subs][1], r, 6);
                c->n_subs++;
            }
        }
    }
    if (o->have[O_ENET_MAC_SEED]) {
        c->random_set = (uint32_t)opt_num(o, O_ENET_MAC_SEED);
        for (int i = 0; i < 6; i++) {
            c->random_mask[i] = (uint8_t)tcpr_random(&c->random_set) % 256;
            for (int j = 0; j < i; j++) {
                if (c->random_mask[i] == c->random_mask[j]) {
                    i--;
                    break;
                }
            }
        }
        if (o->have[O_ENET_MAC_SEED_KEEP_BYTES])
            c->random_keep = (int)opt_num(o, O_ENET_MAC_SEED_KEEP_BYTES);
    }
    if (o->have[O_ENET_DMAC]) {
        int r = dualmac2hex(o->arg[O_ENET_DMAC], c->intf1_dmac, c->intf2_dmac, (int)strlen(o->arg[O_ENET_DMAC]));
        if (r & 1)
            c->mac_mask += MASK_DMAC1;
        if (r & 2)
            c->mac_mask += MASK_DMAC2;
    }
    if (o->have[O_ENET_SMAC]) {
        int r = dualmac2hex(o->arg[O_ENET_SMAC], c->intf1_smac, c->intf2_smac, (int)strlen(o->arg[O_ENET_SMAC]));
        if (r & 1)
            c->mac_mask += MASK_SMAC1;
        if (r & 2)
            c->mac_mask += MASK_SMAC2;
    }
    if (o->have[O_ENET_VLAN]) {
        if (!strcmp(o->arg[O_ENET_VLAN], "add"))
            c->vlan = VLAN_ADD;
        else if (!strcmp(o->arg[O_ENET_VLAN], "del"))
            c->vlan = VLAN_DEL;
        else {
            seterr("Invalid --enet-vlan=%s", o->arg[O_ENET_VLAN]);
            return -1;
        }
        if (c->vlan == VLAN_ADD) {
            if (!o->have[O_ENET_VLAN_TAG]) {
                seterr("Must specify a new 802.1 VLAN tag if vlan mode is add");
                return -1;
            }
            c->vlan_tag = (uint16_t)opt_num(o, O_ENET_VLAN_TAG);
            if (o->have[O_ENET_VLAN_PRI])
                c->vlan_pri = (uint8_t)opt_num(o, O_ENET_VLAN_PRI);
            if (o->have[O_ENET_VLAN_CFI])
                c->vlan_cfi = (uint8_t)opt_num(o, O_ENET_VLAN_CFI);
        }
        if (o->have[O_ENET_VLAN_PROTO]) {
            if (!strcasecmp(o->arg[O_ENET_VLAN_PROTO], "802.1q"))
                c->vlan_proto = ETHERTYPE_VLAN;
            else if (!strcasecmp(o->arg[O_ENET_VLAN_PROTO], "802.1ad"))
                c->vlan_proto = ETHERTYPE_Q_IN_Q;
            else {
                seterr("VLAN protocol \"%s\" is invalid", o->arg[O_ENET_VLAN_PROTO]);
                return -1;
            }
        }
    }
    c->skip_soft_errors = o->have[O_SKIP_SOFT_ERRORS] != 0;
    return 0;
}

static void free_cfg(ocfg_t *c)
{
    if (c->cidrmap2 != c->cidrmap1)
        free(c->cidrmap2);
    free(c->cidrmap1);
    free(c->srcipmap);
    free(c->dstipmap);
    free(c->portmap);
    free(c->subs);
}

/* ------------------------------------------------------------------------- */
/* cache reader: src/common/cache.c:63-140, :321-354                         */
/* ------------------------------------------------------------------------- */
static int parse_cache(const uint8_t *buf, size_t len, const uint8_t **data, uint64_t *num_packets, size_t *data_len)
{
    if (len < 24 || memcmp(buf, "tcpprep\0", 8) != 0) {
        seterr("not a tcpprep cache file");
        return -1;
    }
    if (strtol((const char *)buf + 8, NULL, 10) != 4) {
        seterr("cache file version mismatch");
        return -1;
    }
    uint64_t np = 0;
    for (int i = 0; i < 8; i++)
        np = (np << 8) | buf[12 + i];
    uint16_t ppb = (uint16_t)((buf[20] << 8) | buf[21]);
    uint16_t clen = (uint16_t)((buf[22] << 8) | buf[23]);
    if (ppb == 0) {
        seterr("invalid packets_per_byte");
        return -1;
    }
    uint64_t cache_size = np / ppb + ((np % ppb) ? 1 : 0);
    if (24 + (size_t)clen + cache_size > len) {
        seterr("Cache data length doesn't match cache header");
        return -1;
    }
    *data = buf + 24 + clen;
    *num_packets = np;
    *data_len = (size_t)cache_size;
    return 0;
}

static int check_cache(const uint8_t *cachedata, size_t data_len, uint64_t packetid)
{
    uint64_t index = (packetid - 1) / 4;
    uint32_t bit = (uint32_t)(((packetid - 1) % 4) * 2) + 1;
    /* the reference reads past its buffer here (no bounds check); we read 0 */
    uint8_t byte = index < data_len ? cachedata[index] : 0;
    if (!(byte & (1 << bit)))
        return DIR_NOSEND;
    bit--;
    return (byte & (1 << bit)) ? DIR_C2S : DIR_S2C;
}

/* ------------------------------------------------------------------------- */
/* rewrite driver: src/tcprewrite.c:260-373 over an in-memory pcap           */
/* ------------------------------------------------------------------------- */
static inline uint32_t bswap32_(uint32_t v) { return __builtin_bswap32(v); }

/* Returns 0 on success, -1 on a hard error (output holds the packets written
 * before it, as tcprewrite's exit(-1) leaves it), -2 on bad input/options. */
/* oracle_rewrite_mem over a shard of a capture: `in` holds the file header and a run of
 * whole records whose first is record pkt_base (0-based) of the whole capture, so the
 * tcpprep cache is read at global record numbers (a checker splits a capture of
 * independent records over threads this way; --fuzz-seed and stale reads (Q8) carry
 * state across records and must run unsplit). */
int oracle_rewrite_mem_base(const uint8_t *in, size_t in_len, const uint8_t *cache, size_t cache_len, int argc,
                            const char **argv, uint8_t *out, size_t out_cap, size_t *out_len, int8_t *pkt_status,
                            uint64_t max_status, char *errbuf, int errlen, uint64_t pkt_base)
{
    oopts_t *o = calloc(1, sizeof(oopts_t));
    ocfg_t c;
    int rc = 0;
    uint8_t *buf = NULL;
    const uint8_t *cdata = NULL;
    size_t cdata_len = 0;
    uint64_t cnp = 0;
    size_t op = 0;
    memset(&c, 0, sizeof(c));
    g_err[0] = 0;
    g_warn_count = 0;
    *out_len = 0;

    {   /* the input DLT first: the encoder defaults to the decoder's plugin */
        uint32_t m = 0, lt = 0;
        if (in_len >= 24) {
            memcpy(&m, in, 4);
            memcpy(&lt, in + 20, 4);
            if (m == 0xd4c3b2a1u || m == 0x4d3cb2a1u)
                lt = bswap32_(lt);
        }
        lt &= 0x03ffffff;
        if (lt == 101) /* LINKTYPE_RAW: libpcap's linktype_to_dlt gives DLT_RAW */
            lt = 12;
        static const struct {
            uint32_t dlt;
            int dec;
        } decs[] = {{1, DEC_EN10MB}, {113, DEC_SLL}, {276, DEC_SLL2}, {12, DEC_RAW},  {0, DEC_NULL},
                    {108, DEC_NULL}, {50, DEC_PPP},  {104, DEC_CHDLC}, {178, DEC_JNPR}, {105, DEC_80211},
                    {127, DEC_RADIOTAP}};
        const int ndec = (int)(sizeof(decs) / sizeof(decs[0]));
        int k = 0;
        while (k < ndec && decs[k].dlt != lt)
            k++;
        if (in_len >= 24 && k == ndec) {
            seterr("No DLT plugin available for source DLT: 0x%x (in the oracle's scope)", lt);
            rc = -2;
            goto out;
        }
        c.decoder = k < ndec ? decs[k].dec : DEC_EN10MB;
        c.in_dlt = k < ndec ? (int)lt : 1;
    }
    if (parse_argv(o, argc, argv) < 0 || oracle_post_args(&c, o) < 0) {
        rc = -2;
        goto out;
    }
    if (o->have[O_ENDPOINTS] && !cache) {
        seterr("--endpoints requires a cache file");
        rc = -2;
        goto out;
    }
    if (cache && parse_cache(cache, cache_len, &cdata, &cnp, &cdata_len) < 0) {
        rc = -2;
        goto out;
    }
    if (in_len < 24) {
        seterr("short pcap");
        rc = -2;
        goto out;
    }
    uint32_t magic;
    memcpy(&magic, in, 4);
    int swap = 0, nsec = 0;
    if (magic == 0xa1b2c3d4) {
    } else if (magic == 0xd4c3b2a1) {
        swap = 1;
    } else if (magic == 0xa1b23c4d) {
        nsec = 1;
    } else if (magic == 0x4d3cb2a1) {
        swap = 1;
        nsec = 1;
    } else {
        seterr("bad pcap magic");
        rc = -2;
        goto out;
    }
    /* pcap_open_dead(out_dlt, 65535) + pcap_dump_open header (tcprewrite.c:124,147) */
    if (out_cap < 24) {
        rc = -2;
        goto out;
    }
    {
        /* pcap_dump_open writes dlt_to_linktype(dlt): DLT_RAW (12) is LINKTYPE_RAW (101) */
        const uint32_t olt = c.out_linktype == 12 ? 101u : (uint32_t)c.out_linktype;
        uint32_t hdr[6] = {0xa1b2c3d4u, 0x00040002u, 0, 0, 65535, olt};
        memcpy(out, hdr, 24);
        op = 24;
    }
    buf = calloc(1, MAXPACKET + 65536); /* static pktdata_buff (tcprewrite.c:267-280), zeroed by safe_malloc */
    ostate_t st;
    memset(&st, 0, sizeof(st));
    g_fuzz_state = c.fuzz_seed; /* fuzzing_init (tcprewrite.c:102-103, fuzzing.c:12-20) */
    for (uint64_t k = 0; k < g_fuzz_skip; k++)
        tcpr_random(&g_fuzz_state);
    g_fuzz_draws = 0;
    g_fuzz_factor = c.fuzz_factor ? c.fuzz_factor : 8;
    size_t ip_ = 24;
    uint64_t packetnum = 0;
    while (ip_ + 16 <= in_len) {
        uint32_t rh[4];
        memcpy(rh, in + ip_, 16);
        if (swap)
            for (int k = 0; k < 4; k++)
                rh[k] = bswap32_(rh[k]);
        uint32_t caplen = rh[2], len = rh[3];
        if (ip_ + 16 + caplen > in_len)
            break; /* truncated record: libpcap stops */
        if (caplen > MAX_SNAPLEN)
            break; /* libpcap's reader refuses the record ("invalid packet capture length"):
                      pcap_next returns NULL and tcprewrite's loop ends (tcprewrite.c:289) */
        /* safe_pcap_next (tcprewrite.c:289 -> src/common/utils.c:131-169): a len past
           MAX_SNAPLEN (:136-145) or a zero len or caplen (:147-156) exit(-1)s, so the
           output keeps the records before this one; tcprewrite.c:293-296's errx()s are
           never reached after it */
        if (len > MAX_SNAPLEN) {
            seterr("safe_pcap_next ERROR: Invalid packet length: %u is greater than maximum %u", len, MAX_SNAPLEN);
            rc = -1;
            break;
        }
        if (!len || !caplen) {
            seterr("safe_pcap_next ERROR: Invalid packet length: packet length=%u capture length=%u", len, caplen);
            rc = -1;
            break;
        }
        const size_t file_cap = caplen;
        if (len < caplen) /* utils.c:159-162: caplen = len before the copy and the edit */
            caplen = len;
        uint32_t ts_sec = rh[0], ts_usec = nsec ? rh[1] / 1000 : rh[1];
        packetnum++;
        memcpy(buf, in + ip_ + 16, caplen); /* tcprewrite.c:301: the trimmed caplen */
        ip_ += 16 + file_cap;               /* libpcap moved past the record as stored */
        int dir = DIR_C2S;
        if (cdata)
            dir = check_cache(cdata, cdata_len, pkt_base + packetnum);
        ohdr_t h = {caplen, len};
        int prc = 0, warned = 0;
        if (dir != DIR_NOSEND) {
            prc = oracle_tcpedit_packet(&c, &st, &h, buf, dir, &warned);
            if (prc == TCPEDIT_ERROR) {
                if (pkt_status && packetnum <= max_status)
                    pkt_status[packetnum - 1] = -1;
                rc = -1;
                break;
            }
            if (warned)
                g_warn_count++;
        }
        if (pkt_status && packetnum <= max_status)
            pkt_status[packetnum - 1] = (int8_t)(prc == TCPEDIT_SOFT_ERROR ? -2 : (warned ? 1 : 0));
        if (prc == TCPEDIT_SOFT_ERROR && c.skip_soft_errors)
            continue;
        if (h.caplen) {
            if (op + 16 + h.caplen > out_cap) {
                seterr("output buffer too small");
                rc = -2;
                break;
            }
            uint32_t orh[4] = {ts_sec, ts_usec, h.caplen, h.len};
            memcpy(out + op, orh, 16);
            memcpy(out + op + 16, buf, h.caplen);
            op += 16 + h.caplen;
        }
    }
    *out_len = op;
out:
    if (errbuf && errlen > 0)
        snprintf(errbuf, (size_t)errlen, "%s", g_err);
    free(buf);
    free_cfg(&c);
    free(o);
    return rc;
}

int oracle_rewrite_mem(const uint8_t *in, size_t in_len, const uint8_t *cache, size_t cache_len, int argc,
                       const char **argv, uint8_t *out, size_t out_cap, size_t *out_len, int8_t *pkt_status,
                       uint64_t max_status, char *errbuf, int errlen)
{
    return oracle_rewrite_mem_base(in, in_len, cache, cache_len, argc, argv, out, out_cap, out_len, pkt_status,
                                   max_status, errbuf, errlen, 0);
}

int oracle_warn_count(void) { return g_warn_count; }

/* Exposed for tests: the seed/sequence mixer (parse_args.c:214-230). */
uint64_t oracle_fuzz_draws(void) { return g_fuzz_draws; }
void oracle_set_fuzz_skip(uint64_t draws) { g_fuzz_skip = draws; }

uint32_t oracle_mix_seed(uint32_t seed)
{
    for (int i = 0; i < 5; ++i)
        tcpr_random(&seed);
    return seed;
}

/* Checker helper: cut a capture's records into `parts` byte-balanced runs of whole
 * records (libpcap's stop rules end the walk).  cuts[k] = file offset where run k starts,
 * first[k] = its first record (0-based); cuts[parts] = end of the last whole record.
 * Returns the records walked. */
uint64_t oracle_shard_cuts(const uint8_t *in, size_t in_len, int parts, uint64_t *cuts, uint64_t *first)
{
    uint32_t magic = 0;
    if (in_len >= 4)
        memcpy(&magic, in, 4);
    const int swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    size_t pos = 24, target = in_len > 24 ? (in_len - 24) / (size_t)parts : 0;
    uint64_t n = 0;
    int k = 1;
    cuts[0] = 24;
    first[0] = 0;
    while (pos + 16 <= in_len) {
        while (k < parts && pos >= 24 + target * (size_t)k) {
            cuts[k] = pos;
            first[k] = n;
            k++;
        }
        uint32_t caplen;
        memcpy(&caplen, in + pos + 8, 4);
        if (swap)
            caplen = bswap32_(caplen);
        if (caplen > MAX_SNAPLEN || pos + 16 + caplen > in_len)
            break;
        pos += 16 + caplen;
        n++;
    }
    for (; k <= parts; k++) {
        cuts[k] = pos;
        first[k] = n;
    }
    return n;
}

/* ------------------------------------------------------------------------- */
/* tcpreplay-edit -w <file> [--loop=N] [-K] <tcpedit options> <pcap>         */
/* ------------------------------------------------------------------------- */
/* Returns 0, -1 (a hard error: *out_len = the output up to it), -2 (bad input/options). */
