/*
 * tp_api.c -- host side of the gfx950 tcpprep classification pass
 * (include/tcpprep.h).  Options -> tp_dev_cfg_t, the record walk (what
 * libpcap's pcap_next does for process_raw_packets, src/tcpprep.c:353), one
 * kernel launch (tcpprep_kernels.hip), and the v04 cache header
 * (write_cache, src/common/cache.c:146-219).
 */
#define _GNU_SOURCE
#ifndef __HIP_PLATFORM_AMD__
#define __HIP_PLATFORM_AMD__
#endif
#include <ctype.h>
#include <regex.h>
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "tp_regex.h"
#include "../../../include/tcpprep.h"
#include "tp_dev_cfg.h"

int te_parse_cidr(char *s, te_cidr_t *c); /* te_args.c */

struct tcpprep_hip_s {
    tp_dev_cfg_t cfg;
    int nocomment, has_comment;
    int min_mask, max_mask; /* router mode's --minmask/--maxmask (validated only) */
    uint64_t last_entries;  /* cache entries the last tcpprep_cache_pcap wrote */
    int device;             /* HIP device the classifier runs on (-1: the thread's current one) */
    char comment[8192]; /* the final "args\ncomment" string */
    char errstr[1024];
    uint64_t *mkeys, *mvals; /* --auto over shards: the merged host table (sorted keys) */
    size_t mn;
    int merged;
};

static int tp_err(tcpprep_hip_t *t, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t->errstr, sizeof t->errstr, fmt, ap);
    va_end(ap);
    return -1;
}

int tcpprep_init(tcpprep_hip_t **out)
{
    if (!out)
        return -1;
    tcpprep_hip_t *t = calloc(1, sizeof(*t));
    if (!t)
        return -1;
    for (int p = 0; p <= 1023; p++) { /* tcpprep_api.c:50-53 */
        t->cfg.svc_tcp[p >> 5] |= 1u << (p & 31);
        t->cfg.svc_udp[p >> 5] |= 1u << (p & 31);
    }
    t->cfg.ratio = 2.0; /* --ratio default, tcpprep_opts.def:511-516 */
    t->min_mask = 30;   /* defaults, tcpprep_opts.def:528-552 */
    t->max_mask = 8;
    t->device = -1;
    *out = t;
    return 0;
}

int tcpprep_close(tcpprep_hip_t **t)
{
    if (t && *t) {
        free((*t)->mkeys);
        free((*t)->mvals);
        free(*t);
        *t = NULL;
    }
    return 0;
}

const char *tcpprep_geterr(tcpprep_hip_t *t) { return t ? t->errstr : NULL; }

int64_t tcpprep_last_entries(tcpprep_hip_t *t) { return t ? (int64_t)t->last_entries : -1; }

int tcpprep_set_device(tcpprep_hip_t *t, int device)
{
    if (!t || device < -1)
        return -1;
    t->device = device;
    return 0;
}

int tcpprep_set_pkt_base(tcpprep_hip_t *t, uint64_t pkt_base)
{
    if (!t)
        return -1;
    t->cfg.pkt_base = pkt_base; /* --auto: the shard then needs tcpprep_auto_merge's table */
    return 0;
}

/* parse_cidr(&list, s, ","): cidr.c:244-279 (a ',' list never hides v6 colons) */
static int cidr_list(tcpprep_hip_t *t, const char *arg, te_cidr_t *v, int32_t *n, const char *what)
{
    char buf[4096], *tok = NULL;
    snprintf(buf, sizeof buf, "%s", arg);
    *n = 0;
    for (char *s = strtok_r(buf, ",", &tok); s; s = strtok_r(NULL, ",", &tok)) {
        if (*n >= TP_MAXC)
            return tp_err(t, "%s: more than %d CIDRs", what, TP_MAXC);
        if (!te_parse_cidr(s, &v[(*n)++]))
            return tp_err(t, "Unable to parse %s: %s", what, arg);
    }
    return *n ? 0 : tp_err(t, "Unable to parse %s: %s", what, arg);
}

/* mac2hex (mac.c:37-62): a partial parse keeps the earlier bytes of dst */
static void mac2hex(const char *mac, uint8_t *dst)
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

/* parse_list (list.c:61-130): "^[0-9]+(-([0-9]+|\s*))?$" per ',' token */
static int packet_list(tcpprep_hip_t *t, char *s)
{
    tp_dev_cfg_t *c = &t->cfg;
    char *tok = NULL;
    c->nlist = 0;
    for (char *e = strtok_r(s, ",", &tok); e; e = strtok_r(NULL, ",", &tok)) {
        char *p = e, *second = NULL;
        if (!isdigit((unsigned char)*p))
            return tp_err(t, "Unable to parse: %s", e);
        while (isdigit((unsigned char)*p))
            p++;
        if (*p == '-') {
            *p++ = 0;
            second = p;
            if (isdigit((unsigned char)*p))
                while (isdigit((unsigned char)*p))
                    p++;
            else
                while (isspace((unsigned char)*p))
                    p++;
        }
        if (*p)
            return tp_err(t, "Unable to parse: %s", e);
        if (c->nlist >= TP_MAXC)
            return tp_err(t, "packet list longer than %d ranges", TP_MAXC);
        uint64_t mn = strtoull(e, NULL, 0); /* add_to_list list.c:36-50 */
        c->lmin[c->nlist] = mn;
        c->lmax[c->nlist] = second ? (second[0] ? strtoull(second, NULL, 0) : 0) : mn;
        c->nlist++;
    }
    return c->nlist ? 0 : tp_err(t, "Unable to parse packet list");
}

/* parse_xX_str (xX.c:44-117) for -x/--include and -X/--exclude */
static int include_exclude(tcpprep_hip_t *t, const char *arg, int exclude)
{
    tp_dev_cfg_t *c = &t->cfg;
    char buf[4096];
    snprintf(buf, sizeof buf, "%s", arg);
    if (!buf[0] || buf[1] != ':')
        return tp_err(t, "Syntax error for option %s", exclude ? "--exclude" : "--include");
    int out;
    switch (buf[0]) {
    case 'B': out = TP_XX_BOTH; break;
    case 'D': out = TP_XX_DEST; break;
    case 'E': out = TP_XX_EITHER; break;
    case 'S': out = TP_XX_SOURCE; break;
    case 'P': out = TP_XX_PACKET; break;
    case 'F': return tp_err(t, "BPF include/exclude filters (F:) are not supported");
    default: return tp_err(t, "Invalid include/exclude mode: %c", buf[0]);
    }
    int rc = out == TP_XX_PACKET ? packet_list(t, buf + 2) : cidr_list(t, buf + 2, c->xx_cidr, &c->nxx_cidr, "include/exclude CIDR");
    if (rc < 0)
        return -1;
    c->xx_mode = out + (exclude ? TP_XX_EXCLUDE : 0);
    return 0;
}

/* parse_services (common/services.c:34-93): every line matching "([0-9]+)/(tcp|udp)"
   (REG_ICASE|REG_EXTENDED) marks a server port; the file replaces the 0-1023 default */
static int load_services(tcpprep_hip_t *t, const char *file)
{
    tp_dev_cfg_t *c = &t->cfg;
    FILE *f = fopen(file, "r");
    if (!f)
        return tp_err(t, "Unable to open service file: %s", file);
    regex_t preg;
    if (regcomp(&preg, "([0-9]+)/(tcp|udp)", REG_ICASE | REG_EXTENDED) != 0) {
        fclose(f);
        return tp_err(t, "Unable to compile the services regex");
    }
    memset(c->svc_tcp, 0, sizeof c->svc_tcp);
    memset(c->svc_udp, 0, sizeof c->svc_udp);
    char line[1024]; /* MAXLINE, defines.h.in */
    regmatch_t m[3];
    while (fgets(line, sizeof line, f)) {
        if (regexec(&preg, line, 3, m, 0) != 0)
            continue;
        char port[10] = {0}, proto[10] = {0};
        size_t pl = (size_t)(m[1].rm_eo - m[1].rm_so), ql = (size_t)(m[2].rm_eo - m[2].rm_so);
        memcpy(port, line + m[1].rm_so, pl < 9 ? pl : 9);
        memcpy(proto, line + m[2].rm_so, ql < 9 ? ql : 9);
        uint16_t p = (uint16_t)strtol(port, NULL, 10);
        if (!strcmp(proto, "tcp"))
            c->svc_tcp[p >> 5] |= 1u << (p & 31);
        else if (!strcmp(proto, "udp"))
            c->svc_udp[p >> 5] |= 1u << (p & 31);
    }
    regfree(&preg);
    fclose(f);
    return 0;
}

int tcpprep_parse_args(tcpprep_hip_t *t, int argc, char **argv)
{
    if (!t)
        return -1;
    tp_dev_cfg_t *c = &t->cfg;
    char args[4096] = "";
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i], *eq = strchr(a, '=');
        const char *v = eq ? eq + 1 : NULL;
        size_t nl = eq ? (size_t)(eq - a) : strlen(a);
#define OPT(n) (nl == sizeof(n) - 1 && !strncmp(a, n, nl))
#define NEED_ARG()                                                   \
    do {                                                             \
        if (!v)                                                      \
            return tp_err(t, "option %.*s needs a value", (int)nl, a); \
    } while (0)
        int rc = 0;
        if (OPT("--cidr")) {
            NEED_ARG();
            c->mode = TP_MODE_CIDR;
            rc = cidr_list(t, v, c->cidr, &c->ncidr, "--cidr");
        } else if (OPT("--mac")) {
            NEED_ARG();
            c->mode = TP_MODE_MAC;
            /* macinstring (mac.c:76-115) re-parses the list per packet: resolve it once */
            char buf[4096], *tok = NULL;
            snprintf(buf, sizeof buf, "%s", v);
            uint8_t cur[6] = {0};
            char *s = strtok_r(buf, ",", &tok);
            c->nmac = 0;
            c->mac_first_empty = s == NULL || !*s;
            for (; s && !c->mac_first_empty; s = strtok_r(NULL, ",", &tok)) {
                if (c->nmac >= TP_MAXC)
                    return tp_err(t, "--mac: more than %d addresses", TP_MAXC);
                mac2hex(s, cur);
                memcpy(c->mac[c->nmac++], cur, 6);
            }
        } else if (OPT("--port")) {
            c->mode = TP_MODE_PORT;
        } else if (OPT("--reverse")) {
            c->reverse = 1;
        } else if (OPT("--nonip")) {
            c->nonip = 1; /* DIR_SERVER, tcpprep_opts.def:498 */
        } else if (OPT("--no-arg-comment")) {
            t->nocomment = 1;
        } else if (OPT("--comment")) {
            NEED_ARG();
            snprintf(t->comment, sizeof t->comment, "%s", v);
            t->has_comment = 1;
        } else if (OPT("--include") || OPT("--exclude")) {
            NEED_ARG();
            rc = include_exclude(t, v, OPT("--exclude"));
        } else if (OPT("--auto")) {
            NEED_ARG();
            c->mode = TP_MODE_AUTO; /* tcpprep_opts.def:110-130 */
            if (!strcmp(v, "bridge"))
                c->automode = TP_AUTO_BRIDGE;
            else if (!strcmp(v, "client"))
                c->automode = TP_AUTO_CLIENT;
            else if (!strcmp(v, "server"))
                c->automode = TP_AUTO_SERVER;
            else if (!strcmp(v, "first"))
                c->automode = TP_AUTO_FIRST;
            else if (!strcmp(v, "router"))
                c->automode = TP_AUTO_ROUTER;
            else
                return tp_err(t, "Invalid --auto mode: %s", v);
        } else if (OPT("--minmask") || OPT("--maxmask")) {
            NEED_ARG();
            long m = strtol(v, NULL, 0); /* tcpprep_opts.def:528-552: 0..32 */
            if (m < 0 || m > 32)
                return tp_err(t, "%.*s must be between 0 and 32", (int)nl, a);
            if (OPT("--minmask"))
                t->min_mask = (int)m;
            else
                t->max_mask = (int)m;
        } else if (OPT("--ratio")) {
            NEED_ARG();
            char *end;
            c->ratio = strtod(v, &end); /* tcpprep_api.c:210-216 */
            if (c->ratio < 0)
                return tp_err(t, "Ratio must be a non-negative number");
        } else if (OPT("--services")) {
            NEED_ARG();
            rc = load_services(t, v);
        } else if (OPT("--regex")) {
            NEED_ARG();
            c->mode = TP_MODE_REGEX; /* tcpprep_opts.def:209-231 */
            char e[256];
            if (tp_regex_compile(v, &c->dfa, e, sizeof e) < 0)
                return tp_err(t, "%s", e);
        } else {
            return tp_err(t, "unknown option %s", a);
        }
        if (rc < 0)
            return -1;
        if (!OPT("--comment")) { /* the arg comment leaves out the -C comment (tcpprep_api.c:163-168) */
            strncat(args, a, sizeof args - strlen(args) - 2);
            strcat(args, " ");
        }
#undef OPT
#undef NEED_ARG
    }
    if (!c->mode)
        return tp_err(t, "one of --cidr, --mac, --port, --regex, --auto is required");
    if (t->min_mask <= t->max_mask) /* tcpprep_api.c:204-208 */
        return tp_err(t, "Min network mask len (%d) must be less then max network mask len (%d)", t->min_mask,
                      t->max_mask);
    /* tcpprep_post_args (tcpprep_api.c:160-197): "args\ncomment" */
    char full[sizeof t->comment] = "";
    if (!t->nocomment && args[0]) {
        args[strlen(args) - 1] = 0;
        snprintf(full, sizeof full, "%s", args);
    }
    if (t->has_comment) {
        size_t l = strlen(full);
        if (snprintf(full + l, sizeof full - l, "\n%s", t->comment) >= (int)(sizeof full - l))
            full[sizeof full - 1] = 0; /* (cut at the comment's bound, as the copy below is) */
    }
    memcpy(t->comment, full, sizeof full);
    if (strlen(t->comment) > 65535)
        return tp_err(t, "comment longer than 65535 bytes");
    return 0;
}

size_t tcpprep_cache_bound(tcpprep_hip_t *t, size_t pcap_len)
{
    /* (--auto with --include/--exclude: up to two entries a record, see tcpprep_cache_pcap) */
    return 24 + (t ? strlen(t->comment) : 0) + (pcap_len / 16) / 2 + 1;
}

static uint32_t rd32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

/* check_list (list.c:139-156) */
static int check_list(const tp_dev_cfg_t *c, uint64_t v)
{
    for (int i = 0; i < c->nlist; i++) {
        uint64_t mn = c->lmin[i], mx = c->lmax[i];
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

typedef struct {
    uint64_t *off;
    uint32_t *caplen, *pktnum;
    uint64_t n, records;
} tp_index_t;

/* the record walk: libpcap's pcap_next stops at an oversize or truncated record, and
   safe_pcap_next's rules follow (an exit, or caplen trimmed to len).
   MAC mode leaves records shorter than an Ethernet header out of the cache
   (tcpprep.c:465-468 `break`s before add_cache), so they get no entry -- unless
   the include/exclude packet list, checked first (:362-375), gives them DONT_SEND. */
static int index_pcap(tcpprep_hip_t *t, const uint8_t *img, size_t len, tp_index_t *x)
{
    memset(x, 0, sizeof(*x));
    if (len < 24)
        return tp_err(t, "pcap image too short");
    uint32_t magic;
    memcpy(&magic, img, 4);
    int sw;
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du)
        sw = 0;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u)
        sw = 1;
    else
        return tp_err(t, "not a pcap file (magic 0x%08x)", magic);
    /* the link types tcpprep reads (tcpprep.c:108-125: pcap_datalink, LINKTYPE_RAW as DLT_RAW) */
    uint32_t linktype = rd32(img + 20, sw) & 0x03ffffffu;
    const int dlt = linktype == 101 ? 12 : (int)linktype;
    if (dlt != 1 && dlt != 113 && dlt != 276 && dlt != 12 && dlt != 104 && dlt != 178 && dlt != 50)
        return tp_err(t, "Unsupported pcap DLT type: 0x%x", (unsigned)dlt);
    if (dlt != 1 && t->cfg.mode == TP_MODE_MAC)
        return tp_err(t, "MAC mode splitting is only supported by DLT_EN10MB packet captures.");
    t->cfg.dlt = dlt;
    uint64_t cap = len / 16 + 1;
    x->off = malloc(cap * sizeof(uint64_t));
    x->caplen = malloc(cap * sizeof(uint32_t));
    if (!x->off || !x->caplen)
        return tp_err(t, "out of memory");
    int mac = t->cfg.mode == TP_MODE_MAC, gaps = 0;
    for (size_t off = 24; off + 16 <= len;) {
        const uint32_t fcap = rd32(img + off + 8, sw), plen = rd32(img + off + 12, sw);
        if (fcap > 262144u || off + 16 + fcap > len)
            break;
        /* safe_pcap_next (tcpprep.c:353 -> src/common/utils.c:131-169): a len past
           MAX_SNAPLEN or a zero len or caplen exit(-1)s before write_cache (no cache file);
           len < caplen trims caplen to len */
        if (plen > 262144u || !plen || !fcap)
            return tp_err(t, "safe_pcap_next ERROR: Invalid packet length: packet %llu: packet length=%u capture "
                             "length=%u",
                          (unsigned long long)(x->records + 1), plen, fcap);
        const uint32_t caplen = plen < fcap ? plen : fcap;
        x->records++;
        if (dlt == 178 && caplen >= 4 && !memcmp(img + off + 16, "MGC", 3) && (img[off + 16 + 3] & 0x02))
            /* JUNIPER_FLAG_NO_L2: get_l2len_protocol leaves l2len 0 with l2offset past it, and
               get_ipv4 then forms a pointer ~4 GiB past the packet (get.c:326-344,509-510) */
            return tp_err(t, "record %llu: a Juniper record without an L2 header (the reference reads outside the "
                             "packet there): not served", (unsigned long long)x->records);
        const tp_dev_cfg_t *c = &t->cfg;
        int listed_out = c->nlist && check_list(c, c->pkt_base + x->records) == ((c->xx_mode & TP_XX_EXCLUDE) != 0);
        if (mac && caplen < 14 && !listed_out) {
            if (!gaps) { /* record numbers diverge from entry numbers from here on */
                x->pktnum = malloc(cap * sizeof(uint32_t));
                if (!x->pktnum)
                    return tp_err(t, "out of memory");
                for (uint64_t j = 0; j < x->n; j++)
                    x->pktnum[j] = (uint32_t)(j + 1);
                gaps = 1;
            }
        } else {
            x->off[x->n] = off + 16;
            x->caplen[x->n] = caplen;
            if (gaps)
                x->pktnum[x->n] = (uint32_t)x->records;
            x->n++;
        }
        off += 16 + fcap;
    }
    if (x->records > 0xffffffffull)
        return tp_err(t, "more than 2^32 records");
    return 0;
}

static void index_free(tp_index_t *x)
{
    free(x->off);
    free(x->caplen);
    free(x->pktnum);
}

typedef struct {
    uint8_t *img, *out;
    uint64_t *off;
    uint32_t *caplen, *pktnum;
    tp_dev_cfg_t *cfg;
    tp_tree_t tree;     /* auto modes */
    tp_tree_t *d_tree;  /* its device copy for the classify kernel */
    size_t tree_cap;
} tp_dev_t;

static void dev_free(tp_dev_t *d)
{
    hipFree(d->tree.slots);
    hipFree(d->tree.slot);
    hipFree(d->tree.err);
    hipFree(d->d_tree);
    hipFree(d->img);
    hipFree(d->out);
    hipFree(d->off);
    hipFree(d->caplen);
    hipFree(d->pktnum);
    hipFree(d->cfg);
}

static int stage(tcpprep_hip_t *t, const void *pcap, size_t len, const tp_index_t *x, tp_dev_t *d)
{
    memset(d, 0, sizeof(*d));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return tp_err(t, "no HIP device available: the tcpprep classifier runs on the GPU only");
    if (t->device >= 0 && hipSetDevice(t->device) != hipSuccess)
        return tp_err(t, "hipSetDevice(%d) failed", t->device);
    uint64_t n = x->n ? x->n : 1;
    if (hipMalloc((void **)&d->img, len) != hipSuccess || hipMalloc((void **)&d->out, (n + 3) / 4) != hipSuccess ||
        hipMalloc((void **)&d->off, n * 8) != hipSuccess || hipMalloc((void **)&d->caplen, n * 4) != hipSuccess ||
        hipMalloc((void **)&d->cfg, sizeof(tp_dev_cfg_t)) != hipSuccess ||
        (x->pktnum && hipMalloc((void **)&d->pktnum, n * 4) != hipSuccess)) {
        dev_free(d);
        return tp_err(t, "device allocation failed");
    }
    if (hipMemcpy(d->img, pcap, len, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->off, x->off, x->n * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->caplen, x->caplen, x->n * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->cfg, &t->cfg, sizeof(tp_dev_cfg_t), hipMemcpyHostToDevice) != hipSuccess ||
        (x->pktnum && hipMemcpy(d->pktnum, x->pktnum, x->n * 4, hipMemcpyHostToDevice) != hipSuccess)) {
        dev_free(d);
        return tp_err(t, "host-to-device copy failed");
    }
    if (t->cfg.mode == TP_MODE_AUTO) {
        size_t cap = 1024;
        while (cap < 2 * (t->cfg.automode == TP_AUTO_FIRST ? 2 : 1) * n)
            cap <<= 1;
        d->tree_cap = cap;
        d->tree.mask = cap - 1;
        if (hipMalloc((void **)&d->tree.slots, cap * 16) != hipSuccess ||
            hipMalloc((void **)&d->tree.slot, n * 4) != hipSuccess || hipMalloc((void **)&d->tree.err, 8) != hipSuccess ||
            hipMalloc((void **)&d->d_tree, sizeof(tp_tree_t)) != hipSuccess ||
            hipMemcpy(d->d_tree, &d->tree, sizeof(tp_tree_t), hipMemcpyHostToDevice) != hipSuccess) {
            dev_free(d);
            return tp_err(t, "device allocation failed (host table)");
        }
    }
    return 0;
}

/* the auto modes' first pass (tcpprep.c:480-496 + tree_calculate's inputs): reset the
   table, build it, and report the reference's errx() (packet2tree's len_error) */
static int tree_pass(tcpprep_hip_t *t, const tp_dev_t *d, const tp_index_t *x, const uint8_t *img, hipStream_t st)
{
    size_t cap = d->tree_cap;
    if (hipMemsetAsync(d->tree.slots, 0, cap * 16, st) != hipSuccess ||
        hipMemsetAsync(d->tree.err, 0xff, 8, st) != hipSuccess)
        return tp_err(t, "device memset failed");
    if (tp_launch_tree(d->img, d->off, d->caplen, x->n, d->cfg, t->cfg.automode, t->cfg.pkt_base, d->tree, st) != 0)
        return tp_err(t, "host-table kernel failed");
    uint64_t err = 0;
    if (hipMemcpyAsync(&err, d->tree.err, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return tp_err(t, "host-table kernel failed");
    if (err != ~0ull) /* tree.c:835-837 */
        return tp_err(t, "packet capture length %u too small to process", x->caplen[err]);
    (void)img;
    return 0;
}

/* the merged table's values into this shard's nodes (the local build gave their slots) */
static int apply_merged(tcpprep_hip_t *t, const tp_dev_t *d)
{
    if (!t->merged)
        return 0;
    uint64_t *dk = NULL, *dv = NULL;
    const size_t n = t->mn ? t->mn : 1;
    int rc = -1;
    if (hipMalloc((void **)&dk, n * 8) == hipSuccess && hipMalloc((void **)&dv, n * 8) == hipSuccess &&
        hipMemcpy(dk, t->mkeys, t->mn * 8, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dv, t->mvals, t->mn * 8, hipMemcpyHostToDevice) == hipSuccess &&
        tp_launch_tree_merged(d->tree, d->tree_cap, dk, dv, t->mn, NULL) == 0 && hipDeviceSynchronize() == hipSuccess)
        rc = 0;
    hipFree(dk);
    hipFree(dv);
    return rc < 0 ? tp_err(t, "merged host table upload failed") : 0;
}

int64_t tcpprep_auto_table(tcpprep_hip_t *t, const void *pcap, size_t len, uint64_t *keys, uint64_t *vals, size_t cap)
{
    if (!t || !pcap || (cap && (!keys || !vals)))
        return -1;
    if (t->cfg.mode != TP_MODE_AUTO)
        return tp_err(t, "tcpprep_auto_table needs --auto");
    tp_index_t x;
    if (index_pcap(t, pcap, len, &x) < 0) {
        index_free(&x);
        return -1;
    }
    tp_dev_t d;
    if (stage(t, pcap, len, &x, &d) < 0) {
        index_free(&x);
        return -1;
    }
    int64_t count = -1;
    uint64_t *slots = NULL;
    if (tree_pass(t, &d, &x, pcap, NULL) == 0 && (slots = malloc(d.tree_cap * 16)) &&
        hipMemcpy(slots, d.tree.slots, d.tree_cap * 16, hipMemcpyDeviceToHost) == hipSuccess) {
        count = 0;
        for (size_t s = 0; s < d.tree_cap; s++)
            if (slots[2 * s]) {
                if ((size_t)count < cap) {
                    keys[count] = slots[2 * s];
                    vals[count] = slots[2 * s + 1];
                }
                count++;
            }
    } else if (!t->errstr[0]) {
        tp_err(t, "host table read-back failed");
    }
    free(slots);
    dev_free(&d);
    index_free(&x);
    return count;
}

static int cmp_pair(const void *a, const void *b)
{
    const uint64_t x = ((const uint64_t *)a)[0], y = ((const uint64_t *)b)[0];
    return x < y ? -1 : x > y;
}

int tcpprep_auto_merge(tcpprep_hip_t *t, const uint64_t *keys, const uint64_t *vals, size_t n)
{
    if (!t || (n && (!keys || !vals)))
        return -1;
    if (t->cfg.mode != TP_MODE_AUTO)
        return tp_err(t, "tcpprep_auto_merge needs --auto");
    uint64_t *pr = malloc((n ? n : 1) * 16);
    if (!pr)
        return tp_err(t, "out of memory");
    for (size_t i = 0; i < n; i++) {
        pr[2 * i] = keys[i];
        pr[2 * i + 1] = vals[i];
    }
    qsort(pr, n, 16, cmp_pair);
    free(t->mkeys);
    free(t->mvals);
    t->mkeys = malloc((n ? n : 1) * 8);
    t->mvals = malloc((n ? n : 1) * 8);
    if (!t->mkeys || !t->mvals) {
        free(pr);
        return tp_err(t, "out of memory");
    }
    const int first = t->cfg.automode == TP_AUTO_FIRST;
    size_t m = 0;
    for (size_t i = 0; i < n; i++) {
        const uint64_t k = pr[2 * i], v = pr[2 * i + 1];
        if (m && t->mkeys[m - 1] == k) { /* counts add (their halves stay below 2^32); the
                                            earliest sighting is the largest complement */
            t->mvals[m - 1] = first ? (v > t->mvals[m - 1] ? v : t->mvals[m - 1]) : t->mvals[m - 1] + v;
        } else {
            t->mkeys[m] = k;
            t->mvals[m++] = v;
        }
    }
    free(pr);
    t->mn = m;
    t->merged = 1;
    return 0;
}

int64_t tcpprep_cache_pcap(tcpprep_hip_t *t, const void *pcap, size_t len, void *outv, size_t out_cap)
{
    if (!t || !pcap || !outv)
        return -1;
    tp_index_t x;
    if (index_pcap(t, pcap, len, &x) < 0) {
        index_free(&x);
        return -1;
    }
    if (x.records == 0) { /* tcpprep.c:151-155 */
        index_free(&x);
        return tp_err(t, "No packets were processed.  Filter too limiting?");
    }
    /* --auto with --include/--exclude: the reference's first pass (tcpprep.c:362-375, 413-428)
       adds a DONT_SEND entry for each record a filter drops, and the second pass then adds
       every record's entry after them: the file holds those entries first (the header still
       counts the records).  In the second pass only the filters give DONT_SEND, so they are
       the body's zero entries; the body is shifted by their count below. */
    const int filt_auto = t->cfg.mode == TP_MODE_AUTO && t->cfg.xx_mode;
    if (filt_auto && (t->merged || t->cfg.pkt_base)) {
        index_free(&x);
        return tp_err(t, "--include/--exclude with --auto on shards are not served (the first pass's "
                         "entries of every shard come before the second pass's)");
    }
    size_t clen = strlen(t->comment), hdr = 24 + clen, body = (x.n + 3) / 4;
    /* (--auto with filters: up to one first-pass entry per record before the body) */
    const size_t need = hdr + (filt_auto ? (2 * x.n + 3) / 4 : body);
    if (out_cap < need) {
        index_free(&x);
        return tp_err(t, "cache buffer too small (%zu < %zu)", out_cap, need);
    }
    tp_dev_t d;
    if (stage(t, pcap, len, &x, &d) < 0) {
        index_free(&x);
        return -1;
    }
    uint8_t *out = outv;
    if (t->cfg.mode == TP_MODE_AUTO && t->cfg.pkt_base && !t->merged) {
        dev_free(&d);
        index_free(&x);
        return tp_err(t, "--auto on a shard classifies by the whole capture's host table: "
                         "tcpprep_auto_merge the ranks' tcpprep_auto_table first");
    }
    if (t->cfg.mode == TP_MODE_AUTO && (tree_pass(t, &d, &x, pcap, NULL) < 0 || apply_merged(t, &d) < 0)) {
        dev_free(&d);
        index_free(&x);
        return -1;
    }
    int rc = tp_launch_classify(d.img, d.off, d.caplen, d.pktnum, x.n, d.cfg, d.d_tree, d.out, NULL);
    if (rc == 0 && body && hipMemcpy(out + hdr, d.out, body, hipMemcpyDeviceToHost) != hipSuccess)
        rc = -1;
    if (rc == 0 && hipDeviceSynchronize() != hipSuccess)
        rc = -1;
    dev_free(&d);
    if (rc < 0) {
        index_free(&x);
        return tp_err(t, "classification kernel failed");
    }
    uint64_t entries = x.n;
    if (filt_auto) { /* the first pass's DONT_SEND entries, then the body's */
        uint8_t *b = out + hdr;
        uint64_t f = 0;
        for (uint64_t i = 0; i < x.n; i++)
            f += ((b[i / 4] >> (2 * (i % 4))) & 3u) == 0;
        if (f) {
            memset(b + body, 0, (x.n + f + 3) / 4 - body); /* (the bytes the shift extends into) */
            for (uint64_t i = x.n; i-- > 0;) { /* back to front: the shift moves entries on */
                const unsigned e = (b[i / 4] >> (2 * (i % 4))) & 3u;
                const uint64_t k = i + f;
                b[k / 4] = (uint8_t)((b[k / 4] & ~(3u << (2 * (k % 4)))) | (e << (2 * (k % 4))));
            }
            for (uint64_t k = 0; k < f; k++)
                b[k / 4] &= (uint8_t)~(3u << (2 * (k % 4)));
        }
        entries = x.n + f;
        body = (entries + 3) / 4;
    }
    /* tcpr_cache_file_hdr_t (cache.h:63-72), big-endian counts */
    memcpy(out, "tcpprep\0", 8);
    memcpy(out + 8, "04\0\0", 4);
    for (int i = 0; i < 8; i++)
        out[12 + i] = (uint8_t)(x.records >> (56 - 8 * i));
    out[20] = 0;
    out[21] = 4; /* CACHE_PACKETS_PER_BYTE */
    out[22] = (uint8_t)(clen >> 8);
    out[23] = (uint8_t)clen;
    memcpy(out + 24, t->comment, clen);
    t->last_entries = entries;
    index_free(&x);
    return (int64_t)(hdr + body);
}

int tcpprep_time(tcpprep_hip_t *t, const void *pcap, size_t len, int iters, double *ms_kernel, uint64_t *entries)
{
    if (!t || !pcap || iters <= 0)
        return -1;
    tp_index_t x;
    if (index_pcap(t, pcap, len, &x) < 0) {
        index_free(&x);
        return -1;
    }
    tp_dev_t d;
    if (stage(t, pcap, len, &x, &d) < 0) {
        index_free(&x);
        return -1;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    /* one run = (the auto modes' table reset + build +) the classification */
    int rc = 0;
    for (int i = 0; i <= iters && rc == 0; i++) {
        if (i == 1)
            hipEventRecord(e0, NULL);
        if (t->cfg.mode == TP_MODE_AUTO) {
            size_t cap = d.tree_cap;
            hipMemsetAsync(d.tree.slots, 0, cap * 16, NULL);
            rc = tp_launch_tree(d.img, d.off, d.caplen, x.n, d.cfg, t->cfg.automode, t->cfg.pkt_base, d.tree, NULL);
        }
        if (rc == 0)
            rc = tp_launch_classify(d.img, d.off, d.caplen, d.pktnum, x.n, d.cfg, d.d_tree, d.out, NULL);
    }
    hipEventRecord(e1, NULL);
    float ms = 0;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
        rc = -1;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    dev_free(&d);
    if (ms_kernel)
        *ms_kernel = ms / iters;
    if (entries)
        *entries = x.n;
    index_free(&x);
    return rc < 0 ? tp_err(t, "classification kernel failed") : 0;
}
