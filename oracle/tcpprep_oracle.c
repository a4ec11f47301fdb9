/*
 * tcpprep_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never shipped).
 *
 * A plain-C, single-threaded CPU restatement of tcpprep's per-packet
 * classification pass (src/tcpprep.c:339-587 process_raw_packets) for the
 * per-packet modes -- CIDR (-c), MAC (-e), port (-p) -- with --reverse,
 * --nonip, --comment/--no-arg-comment and the include/exclude filters
 * (-x/-X P:list, S:/D:/B:/E: CIDR), and the cache file writer
 * (src/common/cache.c:146-219 write_cache, :259-314 add_cache), and the auto
 * modes bridge/client/server/first (tree.c:219-565, packet2tree :653-838)
 * with --ratio, and router (whose CIDR build never matches, see tpo_check_tree).
 * Regex mode is not restated (out of scope).
 *
 * Pinning: checked byte-for-byte against the reference's own cache files
 * (test/test.cidr, .cidr_reverse, .mac, .mac_reverse, .port, .comment,
 * .include_packets, .exclude_packets, .include_source, .include_dest, made by
 * and test.auto_{bridge,client,server,first,router}; test/Makefile.am:87-104, from
 * test/test.pcap), committed under tests/golden/,
 * by tests/test_tcpprep.py.
 *
 * It is compiled into the same oracle/_build/liboracle.so as the tcpedit
 * restatement (this file includes it, for the shared L2/L3/L4 locators and the
 * CIDR parser).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 */
#include "tcpedit_oracle.c"
#include <regex.h>

#define TPO_MAXC 64

enum { TPO_CIDR = 1, TPO_MAC = 2, TPO_PORT = 3, TPO_AUTO = 4, TPO_REGEX = 5 };
/* --regex: regcomp(REG_EXTENDED | REG_NOSUB) of the option (tcpprep_opts.def:225) */
static regex_t tpo_re;
static int tpo_re_set;
/* automode: defines.h.in:207 direction_e and tcpprep's BRIDGE/CLIENT/SERVER/FIRST modes */
enum { TPA_BRIDGE = 1, TPA_CLIENT, TPA_SERVER, TPA_FIRST, TPA_ROUTER };
/* xX.h:34-41 */
enum { XX_SOURCE = 1, XX_DEST = 2, XX_BOTH = 4, XX_EITHER = 8, XX_PACKET = 16, XX_EXCLUDE = 128 };

typedef struct {
    int mode, reverse, nonip, nocomment, automode, min_mask, max_mask;
    double ratio;
    ocidr_t cidr[TPO_MAXC];
    int ncidr;
    uint8_t mac[TPO_MAXC][6];
    int nmac, mac_first_empty;
    int xx_mode;               /* 0 = none */
    ocidr_t xx_cidr[TPO_MAXC];
    int nxx_cidr;
    uint64_t lmin[TPO_MAXC], lmax[TPO_MAXC];
    int nlist;
    uint8_t svc_tcp[65536], svc_udp[65536];
    char comment[4096];
    int has_comment;
} tpo_opt_t;

/* parse_cidr(..., ",") cidr.c:244-279 */
static int tpo_cidr_list(ocidr_t *outv, int *n, char *s)
{
    char *tok = NULL, *net;
    *n = 0;
    mask_cidr6(&s, ",");
    net = strtok_r(s, ",", &tok);
    if (!net)
        return 0;
    if (!cidr2cidr(net, &outv[(*n)++]))
        return 0;
    for (;;) {
        if (tok)
            mask_cidr6(&tok, ",");
        net = strtok_r(NULL, ",", &tok);
        if (!net)
            break;
        if (*n >= TPO_MAXC || !cidr2cidr(net, &outv[(*n)++]))
            return 0;
    }
    return 1;
}

/* mac2hex mac.c:37-62: partial parses leave the earlier bytes of `dst` in place */
static void tpo_mac2hex(const char *mac, uint8_t *dst)
{
    while (isspace((unsigned char)*mac))
        mac++;
    for (int i = 0; i < 6; i++) {
        char *pp;
        long l = strtol(mac, &pp, 16);
        if (pp == mac || l > 0xFF || l < 0)
            return;
        if (!(*pp == ':' || (i == 5 && (isspace((unsigned char)*pp) || *pp == '\0'))))
            return;
        dst[i] = (uint8_t)l;
        mac = pp + 1;
    }
}

/* parse_list list.c:61-130 (+ add_to_list :36-50); "^[0-9]+(-([0-9]+|\s*))?$" */
static int tpo_list(tpo_opt_t *o, char *s)
{
    char *tok = NULL;
    for (char *t = strtok_r(s, ",", &tok); t; t = strtok_r(NULL, ",", &tok)) {
        char *p = t;
        if (!isdigit((unsigned char)*p))
            return 0;
        while (isdigit((unsigned char)*p))
            p++;
        char *second = NULL;
        if (*p == '-') {
            *p = 0;
            second = p + 1;
            char *q = second;
            if (isdigit((unsigned char)*q)) {
                while (isdigit((unsigned char)*q))
                    q++;
            } else {
                while (isspace((unsigned char)*q))
                    q++;
            }
            if (*q)
                return 0;
        } else if (*p) {
            return 0;
        }
        if (o->nlist >= TPO_MAXC)
            return 0;
        o->lmin[o->nlist] = strtoull(t, NULL, 0);
        o->lmax[o->nlist] = second ? (second[0] ? strtoull(second, NULL, 0) : 0) : o->lmin[o->nlist];
        o->nlist++;
    }
    return o->nlist > 0;
}

/* parse_xX_str xX.c:44-117 */
static int tpo_xx(tpo_opt_t *o, const char *arg, int exclude)
{
    char buf[4096];
    snprintf(buf, sizeof buf, "%s", arg);
    if (!buf[0] || buf[1] != ':')
        return 0;
    int out;
    switch (buf[0]) {
    case 'B': out = XX_BOTH; break;
    case 'D': out = XX_DEST; break;
    case 'E': out = XX_EITHER; break;
    case 'S': out = XX_SOURCE; break;
    case 'P': out = XX_PACKET; break;
    default: return 0;
    }
    if (out == XX_PACKET) {
        if (!tpo_list(o, buf + 2))
            return 0;
    } else if (!tpo_cidr_list(o->xx_cidr, &o->nxx_cidr, buf + 2)) {
        return 0;
    }
    o->xx_mode = out + (exclude ? XX_EXCLUDE : 0);
    return 1;
}

/* parse_services common/services.c:34-93 */
static int tpo_services(tpo_opt_t *o, const char *file)
{
    FILE *f = fopen(file, "r");
    if (!f)
        return 0;
    regex_t preg;
    if (regcomp(&preg, "([0-9]+)/(tcp|udp)", REG_ICASE | REG_EXTENDED) != 0) {
        fclose(f);
        return 0;
    }
    memset(o->svc_tcp, 0, sizeof o->svc_tcp);
    memset(o->svc_udp, 0, sizeof o->svc_udp);
    char line[1024];
    regmatch_t pm[3];
    while (fgets(line, sizeof line, f)) {
        if (regexec(&preg, line, 3, pm, 0) == 0) {
            char port[16] = {0}, proto[16] = {0};
            int pl = pm[1].rm_eo - pm[1].rm_so, ql = pm[2].rm_eo - pm[2].rm_so;
            strncpy(port, line + pm[1].rm_so, pl < 9 ? pl : 9);
            strncpy(proto, line + pm[2].rm_so, ql < 9 ? ql : 9);
            uint16_t portc = (uint16_t)strtol(port, NULL, 10);
            if (!strcmp(proto, "tcp"))
                o->svc_tcp[portc] = 1;
            else if (!strcmp(proto, "udp"))
                o->svc_udp[portc] = 1;
        }
    }
    regfree(&preg);
    fclose(f);
    return 1;
}

/* option surface: tcpprep_opts.def (long forms only) */
static int tpo_parse(tpo_opt_t *o, int argc, char **argv)
{
    memset(o, 0, sizeof(*o));
    o->ratio = 2.0; /* --ratio default, tcpprep_opts.def:511-516 */
    o->min_mask = 30; /* --minmask / --maxmask defaults, tcpprep_opts.def:528-552 */
    o->max_mask = 8;
    for (int i = 0; i <= 1023; i++) /* tcpprep_init, tcpprep_api.c:50-53 */
        o->svc_tcp[i] = o->svc_udp[i] = 1;
    char args[4096] = "";
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i];
        const char *eq = strchr(a, '=');
        const char *v = eq ? eq + 1 : "";
        size_t nl = eq ? (size_t)(eq - a) : strlen(a);
#define IS(n) (nl == strlen(n) && !strncmp(a, n, nl))
        if (IS("--cidr")) {
            char b[4096];
            snprintf(b, sizeof b, "%s", v);
            o->mode = TPO_CIDR;
            if (!tpo_cidr_list(o->cidr, &o->ncidr, b))
                return -1;
        } else if (IS("--mac")) {
            /* macinstring mac.c:76-115 re-tokenises the string per packet: pre-resolve it */
            char b[4096];
            snprintf(b, sizeof b, "%s", v);
            o->mode = TPO_MAC;
            uint8_t cur[6] = {0};
            char *tok = NULL;
            char *t = strtok_r(b, ",", &tok);
            if (t == NULL || !strlen(t)) {
                o->mac_first_empty = 1;
            } else {
                do {
                    tpo_mac2hex(t, cur);
                    if (o->nmac < TPO_MAXC)
                        memcpy(o->mac[o->nmac++], cur, 6);
                } while ((t = strtok_r(NULL, ",", &tok)) != NULL);
            }
        } else if (IS("--port")) {
            o->mode = TPO_PORT;
        } else if (IS("--regex")) {
            if (tpo_re_set)
                regfree(&tpo_re);
            tpo_re_set = regcomp(&tpo_re, v, REG_EXTENDED | REG_NOSUB) == 0;
            if (!tpo_re_set)
                return -1; /* errx "Unable to compile regex" */
            o->mode = TPO_REGEX;
        } else if (IS("--auto")) {
            o->mode = TPO_AUTO;
            if (!strcmp(v, "bridge"))
                o->automode = TPA_BRIDGE;
            else if (!strcmp(v, "client"))
                o->automode = TPA_CLIENT;
            else if (!strcmp(v, "server"))
                o->automode = TPA_SERVER;
            else if (!strcmp(v, "first"))
                o->automode = TPA_FIRST;
            else if (!strcmp(v, "router"))
                o->automode = TPA_ROUTER;
            else
                return -1;
        } else if (IS("--minmask") || IS("--maxmask")) {
            long m = strtol(v, NULL, 0);
            if (m < 0 || m > 32)
                return -1;
            if (IS("--minmask"))
                o->min_mask = (int)m;
            else
                o->max_mask = (int)m;
        } else if (IS("--ratio")) {
            char *end;
            o->ratio = strtod(v, &end);
            if (o->ratio < 0)
                return -1;
        } else if (IS("--services")) {
            if (!tpo_services(o, v))
                return -1;
        } else if (IS("--reverse")) {
            o->reverse = 1;
        } else if (IS("--nonip")) {
            o->nonip = 1; /* DIR_SERVER (tcpprep_opts.def:498) */
        } else if (IS("--no-arg-comment")) {
            o->nocomment = 1;
        } else if (IS("--comment")) {
            snprintf(o->comment, sizeof o->comment, "%s", v);
            o->has_comment = 1;
        } else if (IS("--include") || IS("--exclude")) {
            if (!tpo_xx(o, v, IS("--exclude")))
                return -1;
        } else {
            return -1;
        }
        if (!IS("--comment")) { /* tcpprep_api.c:160-176 skips -C <comment> */
            strncat(args, a, sizeof args - strlen(args) - 2);
            strcat(args, " ");
        }
#undef IS
    }
    if (!o->mode)
        return -1;
    if (o->min_mask <= o->max_mask)
        return -1; /* tcpprep_api.c:204-208 */
    /* tcpprep_post_args, tcpprep_api.c:160-197: "args\ncomment" */
    char full[8192] = "";
    if (!o->nocomment && args[0]) {
        args[strlen(args) - 1] = 0;
        snprintf(full, sizeof full, "%s", args);
    }
    if (o->has_comment) {
        strcat(full, "\n");
        strncat(full, o->comment, sizeof full - strlen(full) - 1);
    }
    snprintf(o->comment, sizeof o->comment, "%s", full);
    return 0;
}

/* check_list list.c:139-156 */
static int tpo_check_list(const tpo_opt_t *o, uint64_t v)
{
    for (int i = 0; i < o->nlist; i++) {
        uint64_t mn = o->lmin[i], mx = o->lmax[i];
        if (mn != 0 && mx != 0) {
            if (v >= mn && v <= mx)
                return 1;
        } else if (mn == 0) {
            if (v <= mx)
                return 1;
        } else if (v >= mn) {
            return 1;
        }
    }
    return 0;
}

/* check_ip_cidr cidr.c:535-564 / check_ip6_cidr :570-598 over a list */
static int tpo_in4(const ocidr_t *c, int n, uint32_t ip)
{
    if (n == 0)
        return 1;
    for (int i = 0; i < n; i++)
        if (ip_in_cidr(&c[i], ip))
            return 1;
    return 0;
}
static int tpo_in6(const ocidr_t *c, int n, const uint8_t *a)
{
    if (n == 0)
        return 1;
    for (int i = 0; i < n; i++)
        if (ip6_in_cidr(&c[i], a))
            return 1;
    return 0;
}

/* process_xX_by_cidr_ipv4/ipv6 xX.c:124-236: 1 = SEND */
static int tpo_xx_cidr(const tpo_opt_t *o, const uint8_t *ip, int v6)
{
    uint32_t s4 = 0, d4 = 0;
    int s, d;
    if (v6) {
        s = tpo_in6(o->xx_cidr, o->nxx_cidr, ip + 8);
        d = tpo_in6(o->xx_cidr, o->nxx_cidr, ip + 24);
    } else {
        memcpy(&s4, ip + 12, 4);
        memcpy(&d4, ip + 16, 4);
        s = tpo_in4(o->xx_cidr, o->nxx_cidr, s4);
        d = tpo_in4(o->xx_cidr, o->nxx_cidr, d4);
    }
    int m = o->xx_mode & ~XX_EXCLUDE, hit;
    switch (m) {
    case XX_SOURCE: hit = s; break;
    case XX_DEST: hit = d; break;
    case XX_BOTH: hit = d && s; break;
    case XX_EITHER: hit = d || s; break;
    default: return (o->xx_mode & XX_EXCLUDE) ? 0 : 1; /* "Unable to determine action" */
    }
    return (o->xx_mode & XX_EXCLUDE) ? !hit : hit;
}

/* check_dst_port tcpprep.c:211-295: returns 1 (C2S) / 0 (S2C) / nonip */
static int tpo_dst_port(const tpo_opt_t *o, uint8_t *ip, int v6, int len)
{
    uint8_t *end = ip + len, *l4;
    uint8_t proto;
    if (!v6) {
        if (len < ((ip[0] & 0x0f) * 4) + 4)
            return 0;
        proto = ip[9];
        l4 = get_layer4_v4(ip, end);
    } else {
        if (len < 40 + 4)
            return 0;
        proto = get_ipv6_l4proto(ip, end);
        if ((l4 = get_layer4_v6(ip, end)) == NULL)
            return 0;
    }
    if (l4 == NULL)
        return 0;
    if (proto == 6) {
        if (end - l4 < 20)
            return 0;
        return o->svc_tcp[(l4[2] << 8) | l4[3]] ? 1 : 0;
    }
    if (proto == 17) {
        if (end - l4 < 8)
            return 0;
        return o->svc_udp[(l4[2] << 8) | l4[3]] ? 1 : 0;
    }
    return o->nonip;
}

static uint32_t tpo_rd32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

/* tcpprep.c:353's read: libpcap's pcap_next (an oversize or truncated record ends the
 * file), then safe_pcap_next (src/common/utils.c:131-169): len > MAX_SNAPLEN or a zero
 * len or caplen exit(-1)s -- before write_cache (tcpprep.c:194), so no cache is written --
 * and len < caplen trims caplen to len.  Returns 1 with the record's data offset and its
 * (trimmed) caplen, 0 at the end, -5 at the reader's exit; *off moves past the record. */
static int tpo_next(const uint8_t *pcap, size_t len, int sw, size_t *off, size_t *data, uint32_t *caplen)
{
    if (*off + 16 > len)
        return 0;
    const uint32_t cl = tpo_rd32(pcap + *off + 8, sw), pl = tpo_rd32(pcap + *off + 12, sw);
    if (cl > 262144u || *off + 16 + cl > len)
        return 0;
    if (pl > 262144u || !pl || !cl)
        return -5;
    *data = *off + 16;
    *caplen = pl < cl ? pl : cl;
    *off += 16 + cl;
    return 1;
}


/* ---- auto modes: tree.c's host table (RB tree there, open addressing here) ---- */
typedef struct {
    int used, family;
    uint8_t addr[16];
    uint32_t server_cnt, client_cnt;
    int type; /* direction_e: -1 unknown, 0 client, 1 server */
} tpo_node_t;

static tpo_node_t *tpo_nodes;
static size_t tpo_cap;

static tpo_node_t *tpo_find(int family, const uint8_t *addr, int insert, int *inserted)
{
    /* tree_comp (tree.c:590-626) calls ipv6_cmp(&t1->u.ip6, &t1->u.ip6): every IPv6
       address compares equal, so all IPv6 hosts share the first IPv6 node */
    static const uint8_t v6_any[16];
    if (family == 6)
        addr = v6_any;
    int n = family == 4 ? 4 : 16;
    uint64_t h = 1469598103934665603ull ^ (uint64_t)family;
    for (int i = 0; i < n; i++)
        h = (h ^ addr[i]) * 1099511628211ull;
    for (size_t k = 0; k < tpo_cap; k++) {
        tpo_node_t *e = &tpo_nodes[(h + k) & (tpo_cap - 1)];
        if (!e->used) {
            if (!insert)
                return NULL;
            memset(e, 0, sizeof(*e));
            e->used = 1;
            e->family = family;
            memcpy(e->addr, addr, n);
            e->type = -1; /* new_tree(), tree.c:631-644 */
            *inserted = 1;
            return e;
        }
        if (e->family == family && !memcmp(e->addr, addr, n))
            return e;
    }
    return NULL;
}

/* get_l2len_protocol (get.c:263-452) with the capture's datalink, for the DLTs tcpprep
   reads (tcpprep.c:108-118); the IP header is at l2len (get_ipv4/get_ipv6: packet +=
   l2offset, l2len -= l2offset, ip = packet + l2len, get.c:509-510) */
static int tpo_dlt = 1;
static int tpo_l2(const uint8_t *d, uint32_t caplen, uint16_t *proto, uint32_t *l2len)
{
    uint32_t l2off = 0, voff = 0;
    *proto = 0;
    *l2len = 0;
    if (!caplen)
        return -1;
    switch (tpo_dlt) {
    case 12: /* DLT_NULL / DLT_RAW (get.c:287-293): the version nibble, no L2 bytes */
        if ((d[0] >> 4) == 4)
            *proto = 0x0800;
        else if ((d[0] >> 4) == 6)
            *proto = 0x86DD;
        return 0;
    case 178: { /* DLT_JUNIPER_ETHER (get.c:294-345) */
        if (caplen < 4 || memcmp(d, "MGC", 3) != 0)
            return -1;
        if ((d[3] & 0x80) == 0x80) { /* JUNIPER_FLAG_EXT */
            if (caplen < 6)
                return -1;
            l2off = (uint32_t)((d[4] << 8) | d[5]) + 6;
        } else {
            l2off = 4;
        }
        if ((d[3] & 0x02) == 0x02) /* JUNIPER_FLAG_NO_L2: refused before the classification */
            return -1;
        /* fall through to DLT_EN10MB at l2offset (get.c:347-381) */
        uint32_t l2_net_off = 14 + l2off;
        if (caplen <= l2_net_off + 4)
            return -1;
        uint16_t et = (uint16_t)((d[l2off + 12] << 8) | d[l2off + 13]);
        if (parse_metadata(d, caplen, &et, &l2_net_off, &l2off, &voff))
            return -1;
        *l2len = l2_net_off;
        if (et < 1536)
            return -1;
        *proto = et;
        return 0;
    }
    case 50: /* DLT_PPP_SERIAL (get.c:383-400): PPP's IPv4 number counts as IPv4 */
        if (caplen < 4)
            return -1;
        *l2len = 4;
        *proto = (uint16_t)((d[2] << 8) | d[3]) == 0x0021 ? 0x0800 : (uint16_t)((d[2] << 8) | d[3]);
        return 0;
    case 104: /* DLT_C_HDLC (get.c:401-414) */
        if (caplen < 4)
            return -1;
        *l2len = 4;
        *proto = (uint16_t)((d[2] << 8) | d[3]);
        return 0;
    case 113: /* DLT_LINUX_SLL (get.c:415-428): sll_protocol at 14 */
        if (caplen < 16)
            return -1;
        *l2len = 16;
        *proto = (uint16_t)((d[14] << 8) | d[15]);
        return 0;
    case 276: /* DLT_LINUX_SLL2 (get.c:429-442): sll2_protocol first */
        if (caplen < 20)
            return -1;
        *l2len = 20;
        *proto = (uint16_t)((d[0] << 8) | d[1]);
        return 0;
    default: /* DLT_EN10MB */
        return get_l2len_protocol(d, caplen, proto, l2len, &l2off, &voff);
    }
}

/* packet2tree (tree.c:653-838): the node type a packet gives its source; -2 = len_error */
static int tpo_packet2tree(const uint8_t *d, uint32_t caplen)
{
    uint16_t et = 0;
    uint32_t l2len = 0;
    if (tpo_l2(d, caplen, &et, &l2len) == -1)
        return -2;
    long len = caplen, hl = 0;
    uint8_t proto = 0;
    if (et == 0x0800) {
        if (len < (long)l2len + 20)
            return -2;
        proto = d[l2len + 9];
        hl = (d[l2len] & 0x0f) * 4;
    } else if (et == 0x86DD) {
        if (len < (long)l2len + 40)
            return -2;
        proto = d[l2len + 6];
        hl = 40;
    }
    const uint8_t *l4 = d + l2len + hl;
    if (proto == 6) {
        if (len < (long)l2len + 20 + hl)
            return -2;
        uint16_t sport;
        memcpy(&sport, l4, 2);
        if (sport == 20) /* th_sport compared without ntohs */
            return -1;
        if (l4[13] == 0x02)
            return 0; /* SYN: client */
        if (l4[13] == 0x12)
            return 1; /* SYN|ACK: server */
        return -1;
    }
    if (proto == 17) {
        if (len < (long)l2len + 8 + hl)
            return -2;
        uint16_t flags;
        if (((l4[2] << 8) | l4[3]) == 53) {
            if (len < (long)l2len + 8 + 12 + hl)
                return -2;
            memcpy(&flags, l4 + 8 + 2, 2); /* dnsv4_hdr.flags, host order of network bytes */
            return (flags & 0x8000) ? 1 : 0;
        }
        if (((l4[0] << 8) | l4[1]) == 53) {
            if (len < (long)l2len + 8 + 12 + hl)
                return -2;
            memcpy(&flags, l4 + 8 + 2, 2);
            return ((flags & 0x7FFFF) ^ 0x8000) ? 1 : 0;
        }
        return -1;
    }
    if (proto == 1) {
        if (len < (long)l2len + 4 + hl)
            return -2;
        if (l4[0] == 3 && l4[1] == 3)
            return 1; /* port unreachable: source is the server */
    }
    return -1;
}

static uint64_t tpo_pkt_base; /* a shard's first global record number (0-based) */

/* the first pass of auto mode (tcpprep.c:480-496, tree.c:333-538) and tree_calculate
   (tree.c:540-565); returns 0, or -4 on the reference's errx() paths.  The include/exclude
   filters run in this pass too (tcpprep.c:362-375, 413-428): a filtered record adds a
   DONT_SEND entry to the cache here -- before the second pass adds every record's entry
   again -- and stays out of the tree; *dont_send counts those entries. */
static int tpo_tree_pass(const tpo_opt_t *o, const uint8_t *pcap, size_t len, int sw, uint64_t records,
                         uint64_t *dont_send)
{
    *dont_send = 0;
    uint64_t packetnum = 0;
    tpo_cap = 16;
    while (tpo_cap < 4 * records + 16)
        tpo_cap <<= 1;
    free(tpo_nodes);
    tpo_nodes = calloc(tpo_cap, sizeof(tpo_node_t));
    if (!tpo_nodes)
        return -4;
    size_t off = 24, dat = 0;
    uint32_t caplen = 0;
    int nx;
    while ((nx = tpo_next(pcap, len, sw, &off, &dat, &caplen)) != 0) {
        if (nx < 0)
            return -5;
        packetnum++;
        if (o->nlist && !!(o->xx_mode & XX_EXCLUDE) == tpo_check_list(o, tpo_pkt_base + packetnum)) {
            (*dont_send)++;
            continue;
        }
        const uint8_t *d = pcap + dat;
        uint16_t proto = 0;
        uint32_t l2len = 0;
        int res = caplen ? tpo_l2(d, caplen, &proto, &l2len) : -1;
        int v4 = res != -1 && l2len + 20 <= caplen && proto == 0x0800;
        int v6 = !v4 && res != -1 && l2len + 40 <= caplen && proto == 0x86DD;
        if (!v4 && !v6)
            continue;
        if (o->nxx_cidr && o->xx_mode && !tpo_xx_cidr(o, d + l2len, v6)) {
            (*dont_send)++;
            continue;
        }
        int fam = v4 ? 4 : 6, ins = 0;
        const uint8_t *src = d + l2len + (v4 ? 12 : 8), *dst = d + l2len + (v4 ? 16 : 24);
        if (o->automode == TPA_FIRST) { /* add_tree_first_ipv4/ipv6: first sighting wins */
            tpo_node_t *e = tpo_find(fam, src, 1, &ins);
            if (ins) {
                e->type = 0;
                e->client_cnt = 1000;
            }
            ins = 0;
            e = tpo_find(fam, dst, 1, &ins);
            if (ins) {
                e->type = 1;
                e->server_cnt = 1000;
            }
        } else { /* add_tree_ipv4/ipv6 + add_tree_node */
            int t = tpo_packet2tree(d, caplen);
            if (t == -2)
                return -4; /* "packet capture length %d too small to process" */
            tpo_node_t *e = tpo_find(fam, src, 1, &ins);
            if (t == 1)
                e->server_cnt++;
            else if (t == 0)
                e->client_cnt++;
        }
    }
    for (size_t i = 0; i < tpo_cap; i++) { /* tree_calculate */
        tpo_node_t *e = &tpo_nodes[i];
        if (!e->used)
            continue;
        if (e->server_cnt > 0 || e->client_cnt > 0)
            e->type = (double)e->server_cnt >= (double)e->client_cnt * o->ratio ? 1 : 0;
        else
            e->type = -1;
    }
    return 0;
}

/* check_ip_tree / check_ip6_tree (tree.c:219-331): tcpr_dir_t; -4 = unknown system */
static int tpo_check_tree(const tpo_opt_t *o, int fam, const uint8_t *src)
{
    int ins = 0;
    tpo_node_t *e = tpo_find(fam, src, 0, &ins);
    /* router mode: process_tree (tree.c:156-203) builds CIDRs whose family new_cidr()
       leaves 0, so no address is ever "in" them: it succeeds at --maxmask after one
       tree_calculate, and the second pass is check_ip_tree(options->nonip, ...)
       (tcpprep.c:498-509): DIR_CLIENT by default, DIR_SERVER with --nonip */
    int mode = o->automode == TPA_SERVER ? 1 : o->automode == TPA_CLIENT ? 0 : -1;
    if (o->automode == TPA_ROUTER)
        mode = o->nonip ? 1 : 0;
    if (!e && mode == -1)
        return -4;
    if (e && e->type == 1)
        return 2; /* TCPR_DIR_S2C */
    if (e && e->type == 0)
        return 1; /* TCPR_DIR_C2S */
    return mode == 1 ? 2 : mode == 0 ? 1 : -1;
}

/*
 * tcpprep_oracle_run: classify a whole pcap image and write the cache file
 * (header + comment + packed 2-bit entries) into `out`.  Returns the cache
 * size, or -1 on an option error, -2 on a bad pcap, -3 if `cap` is too small,
 * -4 on the reference's errx() paths, -5 when safe_pcap_next exits on a record
 * (tpo_next: no cache is written).
 */
static uint64_t tpo_last_entries;

/* a shard's first global record number (0-based): P: lists keep global numbers */
void tcpprep_oracle_set_pkt_base(uint64_t base) { tpo_pkt_base = base; }
/* cache entries the last tcpprep_oracle_run wrote */
uint64_t tcpprep_oracle_last_entries(void) { return tpo_last_entries; }

long tcpprep_oracle_run(int argc, char **argv, const uint8_t *pcap, size_t len, uint8_t *out, size_t cap)
{
    static tpo_opt_t o;
    if (tpo_parse(&o, argc, argv) < 0)
        return -1;
    if (len < 24)
        return -2;
    uint32_t magic;
    memcpy(&magic, pcap, 4);
    int sw;
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du)
        sw = 0;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u)
        sw = 1;
    else
        return -2;
    /* tcpprep.c:108-125: the link types it reads (LINKTYPE_RAW as DLT_RAW), MAC mode on
       Ethernet only; a Juniper record without an L2 header makes the reference's get_ipv4
       read ~4 GiB past the packet: refused (-4) */
    uint32_t lt = tpo_rd32(pcap + 20, sw) & 0x03ffffffu;
    tpo_dlt = lt == 101 ? 12 : (int)lt;
    if (tpo_dlt != 1 && tpo_dlt != 113 && tpo_dlt != 276 && tpo_dlt != 12 && tpo_dlt != 104 && tpo_dlt != 178 &&
        tpo_dlt != 50)
        return -4; /* errx "Unsupported pcap DLT type" */
    if (tpo_dlt != 1 && o.mode == TPO_MAC)
        return -4; /* err "MAC mode splitting is only supported by DLT_EN10MB packet captures." */
    if (tpo_dlt == 178) {
        size_t off = 24, d = 0;
        uint32_t cl = 0;
        while (tpo_next(pcap, len, sw, &off, &d, &cl) > 0)
            if (cl >= 4 && !memcmp(pcap + d, "MGC", 3) && (pcap[d + 3] & 0x02))
                return -4;
    }
    size_t clen = strlen(o.comment);
    size_t hdr = 24 + clen;
    if (cap < hdr)
        return -3;
    memset(out, 0, cap);
    uint64_t entries = 0;
    if (o.mode == TPO_AUTO) {
        uint64_t recs = 0;
        {
            size_t off = 24, d = 0;
            uint32_t cl = 0;
            while (tpo_next(pcap, len, sw, &off, &d, &cl) > 0)
                recs++;
        }
        const int tr = tpo_tree_pass(&o, pcap, len, sw, recs, &entries); /* (its DONT_SEND entries: zeros) */
        if (tr < 0)
            return tr == -5 ? -5 : -4;
        if (hdr + entries / 4 >= cap && entries)
            return -3;
    }
    uint64_t packetnum = 0;
    static uint8_t pkt[MAXPACKET + 64];
    size_t off = 24, dat = 0;
    uint32_t caplen = 0;
    int nx;
    while ((nx = tpo_next(pcap, len, sw, &off, &dat, &caplen)) != 0) {
        if (nx < 0)
            return -5; /* safe_pcap_next's exit(-1): the cache file stays empty */
        memset(pkt, 0, caplen + 64);
        memcpy(pkt, pcap + dat, caplen);
        packetnum++;
        int send = 1, dir = 0, add = 1; /* dir: 1 = C2S */
        if (o.nlist && !!(o.xx_mode & XX_EXCLUDE) == tpo_check_list(&o, tpo_pkt_base + packetnum)) {
            send = 0; /* tcpprep.c:362-375 */
            goto ADD;
        }
        if (o.mode != TPO_MAC) {
            uint16_t proto = 0;
            uint32_t l2len = 0;
            int res = caplen ? tpo_l2(pkt, caplen, &proto, &l2len) : -1;
            int v4 = res != -1 && l2len + 20 <= caplen && proto == 0x0800;  /* get_ipv4 get.c:483-541 */
            int v6 = !v4 && res != -1 && l2len + 40 <= caplen && proto == 0x86DD; /* get_ipv6 :550-608 */
            if (!v4 && !v6) {
                dir = o.nonip; /* add_cache(SEND, options->nonip) */
                goto ADD;
            }
            uint8_t *ip = pkt + l2len;
            if (o.nxx_cidr && o.xx_mode && !tpo_xx_cidr(&o, ip, v6)) {
                send = 0;
                goto ADD;
            }
            if (o.mode == TPO_AUTO) { /* the second pass: ROUTER/BRIDGE/SERVER/CLIENT/FIRST_MODE cases */
                int r = tpo_check_tree(&o, v6 ? 6 : 4, ip + (v6 ? 8 : 12));
                if (r == -4)
                    return -4; /* "is an unknown system... aborting" */
                dir = r == 1;
            } else if (o.mode == TPO_REGEX) {
                /* check_ipv4_regex / check_ipv6_regex (tcpprep.c:300-335): regexec on
                   inet_ntop's string; the result is 1 or 0, which --reverse turns into 2 or
                   leaves 0 (tcpprep.c:441-442): neither sets the C2S bit */
                char sa[64];
                inet_ntop(v6 ? AF_INET6 : AF_INET, ip + (v6 ? 8 : 12), sa, sizeof sa);
                dir = regexec(&tpo_re, sa, 0, NULL, 0) == 0 && !o.reverse;
            } else if (o.mode == TPO_CIDR) {
                uint32_t s4;
                memcpy(&s4, ip + 12, 4);
                dir = v6 ? tpo_in6(o.cidr, o.ncidr, ip + 8) : tpo_in4(o.cidr, o.ncidr, s4);
                if (o.reverse)
                    dir = !dir;
            } else {
                dir = tpo_dst_port(&o, ip, v6, (int)caplen - (int)l2len);
            }
        } else {
            if (caplen < 14) {
                add = 0; /* tcpprep.c:465-468: `break` before add_cache */
                goto ADD;
            }
            dir = 0;
            if (!o.mac_first_empty)
                for (int m = 0; m < o.nmac; m++)
                    if (!memcmp(pkt + 6, o.mac[m], 6)) {
                        dir = 1;
                        break;
                    }
            if (o.reverse)
                dir = !dir;
        }
    ADD:
        if (add) { /* add_cache cache.c:259-314 */
            size_t byte = hdr + entries / 4;
            if (byte >= cap)
                return -3;
            unsigned bit = (unsigned)(entries % 4) * 2 + 1;
            if (send) {
                out[byte] += (uint8_t)(1u << bit);
                if (dir == 1)
                    out[byte] += (uint8_t)(1u << (bit - 1));
            }
            entries++;
        }
    }
    /* write_cache cache.c:146-219 */
    memcpy(out, "tcpprep\0", 8);
    memcpy(out + 8, "04\0\0", 4);
    for (int i = 0; i < 8; i++)
        out[12 + i] = (uint8_t)(packetnum >> (56 - 8 * i));
    out[20] = 0;
    out[21] = 4;
    out[22] = (uint8_t)(clen >> 8);
    out[23] = (uint8_t)clen;
    memcpy(out + 24, o.comment, clen);
    tpo_last_entries = entries;
    return (long)(hdr + (entries + 3) / 4);
}

#include "tcpreplay_oracle.c"
