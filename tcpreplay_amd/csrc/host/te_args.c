/*
 * te_args.c -- the tcpedit option surface and its one-time derivation into
 * the device tables (te_dev_cfg_t + the port-map LUT).
 *
 * Restates, on the host, the config half of libtcpedit:
 *   tcpedit_post_args         src/tcpedit/parse_args.c:34-254
 *   dlt_en10mb_parse_opts     src/tcpedit/plugins/dlt_en10mb/en10mb.c:226-396
 *   parse_cidr_map/_endpoints src/common/cidr.c:130-418
 *   parse_portmap/ports2PORT  src/tcpedit/portmap.c:55-218
 *   dualmac2hex/mac2hex       src/common/mac.c:33-104
 *   tcpr_random               src/common/utils.c:436-458
 * and the AutoOpts constraints of tcpedit_opts.def / en10mb_opts.def.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "te_internal.h"

const te_optdef_t te_optdefs[OPT__N] = {
    [OPT_PORTMAP] = {"portmap", 'r', 1, 9999, 1},
    [OPT_SEED] = {"seed", 's', 1, 1, 0},
    [OPT_PNAT] = {"pnat", 'N', 1, 2, 1},
    [OPT_SRCIPMAP] = {"srcipmap", 'S', 1, 1, 0},
    [OPT_DSTIPMAP] = {"dstipmap", 'D', 1, 1, 0},
    [OPT_ENDPOINTS] = {"endpoints", 'e', 1, 1, 0},
    [OPT_TCP_SEQUENCE] = {"tcp-sequence", 0, 1, 1, 0},
    [OPT_SKIPBROADCAST] = {"skipbroadcast", 'b', 0, 1, 0},
    [OPT_FIXCSUM] = {"fixcsum", 'C', 0, 1, 0},
    [OPT_FIXHDRLEN] = {"fixhdrlen", 0, 0, 1, 0},
    [OPT_MTU] = {"mtu", 'm', 1, 1, 0},
    [OPT_MTU_TRUNC] = {"mtu-trunc", 0, 0, 1, 0},
    [OPT_EFCS] = {"efcs", 'E', 0, 1, 0},
    [OPT_TTL] = {"ttl", 0, 1, 1, 0},
    [OPT_TOS] = {"tos", 0, 1, 1, 0},
    [OPT_TCLASS] = {"tclass", 0, 1, 1, 0},
    [OPT_FLOWLABEL] = {"flowlabel", 0, 1, 1, 0},
    [OPT_FIXLEN] = {"fixlen", 'F', 1, 1, 0},
    [OPT_FUZZ_SEED] = {"fuzz-seed", 0, 1, 1, 0},
    [OPT_FUZZ_FACTOR] = {"fuzz-factor", 0, 1, 1, 0},
    [OPT_DLT] = {"dlt", 0, 1, 1, 0},
    [OPT_SKIPL2BROADCAST] = {"skipl2broadcast", 0, 0, 1, 0},
    [OPT_ENET_DMAC] = {"enet-dmac", 0, 1, 1, 0},
    [OPT_ENET_SMAC] = {"enet-smac", 0, 1, 1, 0},
    [OPT_ENET_SUBSMAC] = {"enet-subsmac", 0, 1, 9999, 1},
    [OPT_ENET_MAC_SEED] = {"enet-mac-seed", 0, 1, 1, 0},
    [OPT_ENET_MAC_SEED_KEEP_BYTES] = {"enet-mac-seed-keep-bytes", 0, 1, 1, 0},
    [OPT_ENET_VLAN] = {"enet-vlan", 0, 1, 1, 0},
    [OPT_ENET_VLAN_TAG] = {"enet-vlan-tag", 0, 1, 1, 0},
    [OPT_ENET_VLAN_CFI] = {"enet-vlan-cfi", 0, 1, 1, 0},
    [OPT_ENET_VLAN_PRI] = {"enet-vlan-pri", 0, 1, 1, 0},
    [OPT_ENET_VLAN_PROTO] = {"enet-vlan-proto", 0, 1, 1, 0},
    [OPT_SKIP_SOFT_ERRORS] = {"skip-soft-errors", 0, 0, 1, 0},
    [OPT_USER_DLT] = {"user-dlt", 0, 1, 1, 0},
    [OPT_USER_DLINK] = {"user-dlink", 0, 1, 2, 1},
    [OPT_HDLC_CONTROL] = {"hdlc-control", 0, 1, 1, 0},
    [OPT_HDLC_ADDRESS] = {"hdlc-address", 0, 1, 1, 0},
};

void te_seterr(tcpedit_t *t, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t->pub.runtime.errstr, sizeof(t->pub.runtime.errstr), fmt, ap);
    va_end(ap);
}

void te_setwarn(tcpedit_t *t, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t->pub.runtime.warnstr, sizeof(t->pub.runtime.warnstr), fmt, ap);
    va_end(ap);
}

/* ISO C rand_r extended to 32 bits (utils.c:436-458) */
uint32_t te_tcpr_random(uint32_t *seed)
{
    uint32_t n = *seed, r;
    n = n * 1103515245u + 12345u;
    r = (uint32_t)((int)(n / 65536) % 2048);
    n = n * 1103515245u + 12345u;
    r = (r << 10) ^ (uint32_t)((int)(n / 65536) % 1024);
    n = n * 1103515245u + 12345u;
    r = (r << 10) ^ (uint32_t)((int)(n / 65536) % 1024);
    *seed = n;
    return r;
}

/* ------------------------------------------------------------------------- */
/* option store                                                              */
/* ------------------------------------------------------------------------- */
static int find_long(const char *name, size_t n)
{
    for (int k = 0; k < OPT__N; k++)
        if (strlen(te_optdefs[k].name) == n && strncmp(te_optdefs[k].name, name, n) == 0)
            return k;
    return -1;
}

static int store(tcpedit_t *t, int k, const char *value)
{
    const te_optdef_t *d = &te_optdefs[k];
    if (d->has_arg && !value) {
        te_seterr(t, "option --%s requires an argument", d->name);
        return -1;
    }
    if (d->stacked) {
        if (t->nstack[k] >= d->max || t->nstack[k] >= TE_MAX_STACK) {
            te_seterr(t, "too many --%s options (max %d)", d->name, d->max);
            return -1;
        }
        t->stack[k][t->nstack[k]++] = strdup(value);
    } else if (t->have[k]) {
        te_seterr(t, "option --%s may appear only once", d->name);
        return -1;
    }
    t->have[k] = 1;
    t->opt_src |= TE_SRC_STORE;
    free(t->arg[k]);
    t->arg[k] = value ? strdup(value) : NULL;
    t->post_args_done = 0;
    return 0;
}

int tcpedit_set_option(tcpedit_t *t, const char *name, const char *value)
{
    if (!t || !name)
        return -1;
    while (*name == '-')
        name++;
    int k = find_long(name, strlen(name));
    if (k < 0) {
        te_seterr(t, "unknown tcpedit option --%s", name);
        return -1;
    }
    return store(t, k, value);
}

int tcpedit_parse_args(tcpedit_t *t, int argc, char **argv, int *unused)
{
    int nun = 0;
    if (!t)
        return -1;
    t->opt_src |= TE_SRC_STORE; /* even an empty command line is an option source */
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i];
        int k = -1;
        const char *val = NULL;
        if (a[0] == '-' && a[1] == '-' && a[2]) {
            const char *eq = strchr(a + 2, '=');
            k = find_long(a + 2, eq ? (size_t)(eq - (a + 2)) : strlen(a + 2));
            if (k >= 0 && te_optdefs[k].has_arg) {
                if (eq)
                    val = eq + 1;
                else if (i + 1 < argc)
                    val = argv[++i];
            }
        } else if (a[0] == '-' && a[1] && !a[2]) {
            for (int j = 0; j < OPT__N; j++)
                if (te_optdefs[j].shortopt == a[1])
                    k = j;
            if (k >= 0 && te_optdefs[k].has_arg && i + 1 < argc)
                val = argv[++i];
        }
        if (k < 0) {
            if (unused)
                unused[nun] = i;
            nun++;
            continue;
        }
        if (store(t, k, val) < 0)
            return -1;
    }
    return nun;
}

/* ------------------------------------------------------------------------- */
/* CIDR parsing (cidr.c:130-418)                                             */
/* ------------------------------------------------------------------------- */
static int parse_one_cidr(char *s, te_cidr_t *c)
{
    unsigned int o[4];
    memset(c, 0, sizeof(*c));
    c->masklen = 99; /* new_cidr() default (cidr.c:103) */
    for (char *p = s; *p; ++p) {
        if (*p == '#')
            *p = ':';
        else if (*p == ']') {
            *p = 0;
            break;
        }
    }
    int n = sscanf(s, "%u.%u.%u.%u/%d", &o[0], &o[1], &o[2], &o[3], &c->masklen);
    if (n == 4 || n == 5) {
        if (n == 4)
            c->masklen = 32;
        if (c->masklen > 32)
            return 0;
        for (int i = 0; i < 4; i++)
            if (o[i] > 255)
                return 0;
        uint8_t b[4] = {(uint8_t)o[0], (uint8_t)o[1], (uint8_t)o[2], (uint8_t)o[3]};
        memcpy(&c->network, b, 4); /* inet_aton: network byte order */
        c->family = 4;
        return 1;
    }
    char *slash = strchr(s, '/');
    if (slash) {
        *slash = 0;
        sscanf(slash + 1, "%d", &c->masklen);
    } else {
        c->masklen = 128;
    }
    if (c->masklen < 0 || c->masklen > 128)
        return 0;
    if (*s == '[')
        s++;
    if (inet_pton(AF_INET6, s, c->network6) <= 0)
        return 0;
    c->family = 6;
    return 1;
}

/* mask_cidr6 (cidr.c:223-236): inside a leading "[...]" turn ':' into '#' */
static void hide_v6_colons(char **p)
{
    if (**p == '[') {
        ++*p;
        for (char *q = *p; *q && *q != ']'; ++q)
            if (*q == ':')
                *q = '#';
    }
}

/* one "from:to" element -> pair; returns 1 ok, 0 not a pair, -1 bad CIDR */
static int parse_pair(char *piece, te_cidrmap_t *m)
{
    char *save = NULL, *tok;
    te_cidr_t tmp[2];
    int n = 0;
    hide_v6_colons(&piece);
    tok = strtok_r(piece, ":", &save);
    while (tok) {
        if (n < 2 && !parse_one_cidr(tok, &tmp[n]))
            return -1;
        if (n >= 2) { /* extra elements are parsed (and validated) then ignored */
            te_cidr_t junk;
            if (!parse_one_cidr(tok, &junk))
                return -1;
        }
        n++;
        if (save)
            hide_v6_colons(&save);
        tok = strtok_r(NULL, ":", &save);
    }
    if (n < 2)
        return 0;
    m->from = tmp[0];
    m->to = tmp[1];
    return 1;
}

/* the map a parse fills (cfg.cidr_spill order: cidrmap1, cidrmap2, srcipmap, dstipmap) */
static int cmap_which(tcpedit_t *t, const te_cidrmap_t *out)
{
    return out == t->cfg.cidrmap1 ? 0 : out == t->cfg.cidrmap2 ? 1 : out == t->cfg.srcipmap ? 2 : 3;
}

/* parse_cidr_map (cidr.c:380-418): the list is unbounded; its first TE_MAX_CIDRMAP pairs
   go inline into the config, the rest into the context's spill list (on the device with
   the config) */
static int parse_cidr_map(tcpedit_t *t, const char *arg, te_cidrmap_t *out, int32_t *nout, const char *what)
{
    char *s = strdup(arg), *save = NULL;
    int n = 0, ok = 1, cap = 0;
    const int w = cmap_which(t, out);
    free(t->cspill[w]);
    t->cspill[w] = NULL;
    for (char *piece = strtok_r(s, ",", &save); piece; piece = strtok_r(NULL, ",", &save)) {
        te_cidrmap_t m;
        int rc = parse_pair(piece, &m);
        if (rc > 0) {
            if (n < TE_MAX_CIDRMAP) {
                out[n] = m;
            } else {
                if (n - TE_MAX_CIDRMAP >= cap) {
                    cap = cap ? 2 * cap : 16;
                    te_cidrmap_t *g = realloc(t->cspill[w], sizeof(te_cidrmap_t) * (size_t)cap);
                    if (!g) {
                        te_seterr(t, "out of memory");
                        ok = 0;
                        break;
                    }
                    t->cspill[w] = g;
                }
                t->cspill[w][n - TE_MAX_CIDRMAP] = m;
            }
        }
        if (rc < 0) {
            te_seterr(t, "Unable to parse as a valid CIDR: %s", piece);
            ok = 0;
            break;
        }
        if (rc == 0) {
            te_seterr(t, "Unable to parse %s=%s", what, arg);
            ok = 0;
            break;
        }
        n++;
    }
    if (ok && n == 0) {
        te_seterr(t, "Unable to parse %s=%s", what, arg);
        ok = 0;
    }
    free(s);
    *nout = n;
    return ok;
}

/* parse_endpoints (cidr.c:290-362): -e A:B == -N 0.0.0.0/0:A -N 0.0.0.0/0:B */
static int parse_endpoints(tcpedit_t *t, const char *arg)
{
    char buf[256];
    char *s = strdup(arg);
    int ok = 0;
    if (*s == '[') {
        char *p = strstr(s, "]:[");
        if (p) {
            *p = 0;
            snprintf(buf, sizeof(buf), "[::/0]:%s]", s);
            if (parse_cidr_map(t, buf, t->cfg.cidrmap1, &t->cfg.n_cidrmap1, "--endpoints")) {
                snprintf(buf, sizeof(buf), "[::/0]:%s", p + 2);
                ok = parse_cidr_map(t, buf, t->cfg.cidrmap2, &t->cfg.n_cidrmap2, "--endpoints");
            }
        }
    } else {
        char *save = NULL, *a = strtok_r(s, ":", &save), *b = a ? strtok_r(NULL, ":", &save) : NULL;
        if (a && b) {
            snprintf(buf, sizeof(buf), "0.0.0.0/0:%s", a);
            if (parse_cidr_map(t, buf, t->cfg.cidrmap1, &t->cfg.n_cidrmap1, "--endpoints")) {
                snprintf(buf, sizeof(buf), "0.0.0.0/0:%s", b);
                ok = parse_cidr_map(t, buf, t->cfg.cidrmap2, &t->cfg.n_cidrmap2, "--endpoints");
            }
        }
    }
    free(s);
    return ok;
}

/* ------------------------------------------------------------------------- */
/* port map -> first-match LUT (portmap.c:55-260)                            */
/* ------------------------------------------------------------------------- */
typedef struct {
    long from, to;
} pm_ent_t;

static int pm_push(pm_ent_t **v, int *n, int *cap, long from, long to)
{
    if (*n == *cap) {
        *cap = *cap ? *cap * 2 : 64;
        *v = realloc(*v, sizeof(pm_ent_t) * (size_t)*cap);
    }
    (*v)[(*n)++] = (pm_ent_t){from, to};
    return 1;
}

static long strict_long(const char *s, int *bad)
{
    char *end;
    long v = strtol(s, &end, 10);
    *bad = *end != '\0';
    return v;
}

/* ports2PORT: one "<ports>:<port>" record; appends its chain (0 = syntax error) */
static int pm_record(char *rec, pm_ent_t **v, int *n, int *cap)
{
    char *save = NULL, *from_s = strtok_r(rec, ":", &save), *to_s = strtok_r(NULL, ":", &save);
    int bad;
    if (strtok_r(NULL, ":", &save) || !from_s || !to_s)
        return 0;
    if (strchr(from_s, '-') && strchr(from_s, '+'))
        return 0;
    long to = strict_long(to_s, &bad);
    if (bad || to < 0 || to > 65535)
        return 0;
    uint16_t to_n = htons((uint16_t)to);
    if (strchr(from_s, '-')) {
        char *s2 = NULL, *b = strtok_r(from_s, "-", &s2), *e = strtok_r(NULL, "-", &s2);
        if (!b || !e)
            return 0;
        long lb = strict_long(b, &bad);
        if (bad)
            return 0;
        long le = strtol(e, NULL, 10);
        if (lb < 0 || lb > 65535 || le < 0 || le > 65535)
            return 0;
        for (long i = lb; i <= le; i++)
            pm_push(v, n, cap, htons((uint16_t)i), to_n);
        pm_push(v, n, cap, 0, 0); /* the zeroed trailing node (portmap.c:117-124) */
    } else if (strchr(from_s, '+')) {
        int start = *n;
        char *s2 = NULL;
        char *p = strtok_r(from_s, "+", &s2);
        long f = strict_long(p, &bad);
        if (bad)
            return 0;
        pm_push(v, n, cap, htons((uint16_t)f), to_n);
        while ((p = strtok_r(NULL, "+", &s2)) != NULL) {
            f = strict_long(p, &bad);
            if (bad || f < 0 || f > 65535) {
                *n = start;
                return 0;
            }
            pm_push(v, n, cap, htons((uint16_t)f), to_n);
        }
    } else {
        long f = strict_long(from_s, &bad);
        if (bad || f < 0 || f > 65535)
            return 0;
        pm_push(v, n, cap, htons((uint16_t)f), to_n);
    }
    return 1;
}

/* parse_portmap: the first record must parse; later bad records are dropped */
static int pm_parse(const char *arg, pm_ent_t **v, int *n, int *cap)
{
    char *s = strdup(arg), *save = NULL;
    char *rec = strtok_r(s, ",", &save);
    int ok = rec && pm_record(rec, v, n, cap);
    if (ok)
        while ((rec = strtok_r(NULL, ",", &save)) != NULL)
            pm_record(rec, v, n, cap);
    free(s);
    return ok;
}

/* ------------------------------------------------------------------------- */
/* MAC strings (mac.c:33-104)                                                */
/* ------------------------------------------------------------------------- */
static void mac_from_str(const char *m, uint8_t *dst)
{
    char *end;
    while (isspace((unsigned char)*m))
        m++;
    for (int i = 0; i < 6; i++) {
        long l = strtol(m, &end, 16);
        if (end == m || l < 0 || l > 0xff)
            return;
        if (!(*end == ':' || (i == 5 && (isspace((unsigned char)*end) || *end == '\0'))))
            return;
        dst[i] = (uint8_t)l;
        m = end + 1;
    }
}

static int dual_mac(const char *arg, uint8_t *first, uint8_t *second)
{
    int ret = 0;
    if (strlen(arg) <= 1)
        return 0;
    char *s = strdup(arg), *save = NULL;
    char *a = strtok_r(s, ",", &save);
    if (a && *a) {
        mac_from_str(a, first);
        ret = 1;
    }
    char *b = strtok_r(NULL, ",", &save);
    if (b && *b) {
        mac_from_str(b, second);
        ret += 2;
    }
    free(s);
    return ret;
}

/* read_hexstring (src/common/utils.c:331-380): comma-separated hex bytes, strtol base
 * 16; -1 where the reference errx()s (no byte, or a byte > 0xff) */
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

/* ------------------------------------------------------------------------- */
/* derivation                                                                */
/* ------------------------------------------------------------------------- */
static int num_arg(tcpedit_t *t, int k, long lo, long hi, long *out)
{
    char *end;
    long v = strtol(t->arg[k], &end, 0);
    if (*end != '\0' || end == t->arg[k]) {
        te_seterr(t, "invalid number for --%s: %s", te_optdefs[k].name, t->arg[k]);
        return 0;
    }
    if (v < lo || v > hi) {
        te_seterr(t, "--%s value %ld out of range [%ld, %ld]", te_optdefs[k].name, v, lo, hi);
        return 0;
    }
    *out = v;
    return 1;
}

static int conflict(tcpedit_t *t, int a, int b)
{
    if (t->have[a] && t->have[b]) {
        te_seterr(t, "--%s cannot be combined with --%s", te_optdefs[a].name, te_optdefs[b].name);
        return 1;
    }
    return 0;
}

static int requires_(tcpedit_t *t, int a, int b)
{
    if (t->have[a] && !t->have[b]) {
        te_seterr(t, "--%s requires --%s", te_optdefs[a].name, te_optdefs[b].name);
        return 1;
    }
    return 0;
}

/* the LUT's non-identity entries, for the wave lane's LDS lookup (te_dev_cfg.h n_pm) */
static void pm_sparse(tcpedit_t *t)
{
    te_dev_cfg_t *c = &t->cfg;
    c->n_pm = 0;
    for (int p = 0; t->portlut && p < 65536; p++) {
        if (t->portlut[p] == p)
            continue;
        if (c->n_pm == TE_MAX_PM) {
            c->n_pm = -1;
            return;
        }
        c->pm_from[c->n_pm] = (uint16_t)p;
        c->pm_to[c->n_pm++] = t->portlut[p];
    }
}

/* the decoder plugin of an input DLT (tcpedit_dlt_init, dlt_plugins.c:115-160; the
 * plugins' dlt_value): -1 when this build has none */
int te_decoder_of(int dlt)
{
    switch (dlt) {
    case 1: return TE_DEC_EN10MB;
    case 113: return TE_DEC_SLL;   /* DLT_LINUX_SLL */
    case 276: return TE_DEC_SLL2;  /* DLT_LINUX_SLL2 */
    case 12: return TE_DEC_RAW;    /* DLT_RAW */
    case 0:                        /* DLT_NULL */
    case 108: return TE_DEC_NULL;  /* DLT_LOOP (loop.c: dlt_null's functions) */
    case 50: return TE_DEC_PPP;    /* DLT_PPP_SERIAL (pppserial.c:41) */
    case 104: return TE_DEC_CHDLC; /* DLT_C_HDLC */
    case 178: return TE_DEC_JNPR;  /* DLT_JUNIPER_ETHER (jnpr_ether.c:44) */
    case 105: return TE_DEC_80211; /* DLT_IEEE802_11 (ieee80211.c:38) */
    case 127: return TE_DEC_RADIOTAP; /* DLT_IEEE802_11_RADIO (radiotap.c:32) */
    default: return -1;
    }
}

/* the decoder's own plugin as the encoder (no --dlt) */
int te_default_encoder(int dec)
{
    switch (dec) {
    case TE_DEC_EN10MB: return TE_ENC_EN10MB;
    case TE_DEC_PPP: return TE_ENC_PPP;
    case TE_DEC_CHDLC: return TE_ENC_HDLC;
    default: return TE_ENC_NOENC;
    }
}

/* the decoded L2 header's length (the encoders replace it): en10mb's varies (14 assumed
 * for the slot headroom; VLAN/MPLS make it longer, never shorter) */
int te_decoder_l2len(int dec)
{
    switch (dec) {
    case TE_DEC_SLL: return 16;
    case TE_DEC_SLL2: return 20;
    case TE_DEC_RAW: return 0;
    case TE_DEC_NULL:
    case TE_DEC_PPP:
    case TE_DEC_CHDLC: return 4;
    case TE_DEC_JNPR: return 6;      /* the 6-byte Juniper header alone: a frame whose extensions
                                        are not Ethernet (TCPEDIT_WARN) decodes to just it */
    case TE_DEC_80211: return 24;    /* ieee80211_hdr_t, at least */
    case TE_DEC_RADIOTAP: return 24; /* (never encoded: every record is a soft error) */
    default: return 14;
    }
}

/* the decoder/encoder pairs this build does not serve, refused loudly, and the Q18
 * carry flag.  s2c: records may be S2C (a tcpprep cache, or tcpedit_packet's caller). */
int te_check_decoder_cfg(tcpedit_t *t, int s2c)
{
    te_dev_cfg_t *c = &t->cfg;
    const int foreign = c->decoder != TE_DEC_EN10MB;
    const int eth_addr = c->decoder == TE_DEC_EN10MB || TE_DEC_ETH_ADDR(c->decoder);
    c->l2carry = TE_DEC_ETH_ADDR(c->decoder) && c->encoder == TE_ENC_EN10MB &&
                 !(c->mac_mask & TE_MASK_DMAC1);
    /* (served: --enet-vlan=add behind another decoder -- the tag lands at the decoder extra's
       never-set vlan_offset 0, en10mb.c:696-715 -- and a decoder without Ethernet addresses
       into --dlt=enet without both MACs -- every packet fails after the encoder's memmove and
       is written half-moved, en10mb.c:567-619: edit_pkt.hpp en10mb_encode_foreign) */
    (void)foreign;
    (void)eth_addr;
    (void)s2c;
    /* --fuzz-seed behind any decoder and into any encoder: a fuzzed record goes back to
       `again:` and is decoded by the input decoder and encoded a second time (tcpedit.c:89,
       250-258); the slot headroom holds both encodes (te_slot_head).  With the en10mb
       encoder's dst_modified carry the second encode writes the carry too: its
       mark runs the edit itself (te_launch_edit, LaunchArgs.q18_keys) */
    return 0;
}

/* tcpedit_init (tcpedit.c:371-403), dlt_en10mb_init (en10mb.c:117-122) and the
 * encoder defaults of tcpedit_dlt_post_args (dlt_plugins.c:178-183: the decoder's) */
void te_cfg_defaults(te_dev_cfg_t *c, int dlt)
{
    memset(c, 0, sizeof(*c));
    c->mtu = 1500; /* DEFAULT_MTU (tcpedit.c:382) */
    c->tos = c->tclass = c->flowlabel = -1;
    c->vlan_tag = 65535; /* en10mb.c:117-122 */
    c->vlan_pri = 255;
    c->vlan_cfi = 255;
    c->vlan_proto = 0x8100;
    c->decoder = te_decoder_of(dlt);
    c->encoder = te_default_encoder(c->decoder);
    c->out_linktype = dlt;
    c->user_length = -1;
    c->hdlc_address = c->hdlc_control = 65535;
    c->fuzz_factor = 8; /* DEFAULT_FUZZ_FACTOR */
}

/* the DLT plugin ids of the encoders this build carries (plugins/dlt_*): the user
 * plugin answers for DLT_USER0 (user.c:40), hdlc for DLT_C_HDLC (hdlc.c:40) */
static int encoder_dlt(const tcpedit_t *t, int enc)
{
    if (enc == TE_ENC_USER)
        return 147;
    if (enc == TE_ENC_HDLC)
        return 104;
    if (enc == TE_ENC_PPP)
        return 50;
    if (enc == TE_ENC_NOENC)
        return t->cfg.out_linktype; /* the non-encoding plugin named (or the decoder's own) */
    return 1;
}

void te_sync_pub(tcpedit_t *t)
{
    tcpedit_ref_t *p = &t->pub;
    const te_dev_cfg_t *c = &t->cfg;
    p->dlt_ctx = &t->dltc;
    t->dltc.tcpedit = t;
    t->dltc.decoder_dlt = t->dlt;
    t->dltc.encoder_dlt = encoder_dlt(t, c->encoder);
    p->skip_broadcast = c->skip_broadcast != 0;
    p->fixlen = (tcpedit_fixlen)c->fixlen;
    p->editdir = TCPEDIT_EDIT_BOTH;
    p->rewrite_ip = c->rewrite_ip != 0;
    p->tcp_sequence_enable = c->tcp_sequence_enable;
    p->tcp_sequence_adjust = c->tcp_sequence_adjust;
    p->fixcsum = c->fixcsum != 0;
    p->efcs = c->efcs != 0;
    p->ttl_mode = (tcpedit_ttl_mode)c->ttl_mode;
    p->ttl_value = (uint8_t)c->ttl_value;
    p->tos = c->tos;
    p->flowlabel = c->flowlabel;
    p->tclass = c->tclass;
    p->seed = c->seed;
    p->mtu = c->mtu;
    p->mtu_truncate = c->mtu_truncate != 0;
    p->fuzz_seed = t->fuzz_seed;
    p->fuzz_factor = t->fuzz_factor;
    p->fixhdrlen = c->fixhdrlen != 0;
}

/* fuzzing_init (fuzzing.c:12-20): the process-wide seed and factor, applied to every
 * context's device state before its next edit (te_upload_cfg) */
uint64_t te_fuzz_init_gen;
uint32_t te_fuzz_init_seed, te_fuzz_init_factor;

void fuzzing_init(uint32_t fuzz_seed, uint32_t fuzz_factor)
{
    if (!fuzz_factor) { /* assert(_fuzz_factor) */
        fprintf(stderr, "fuzzing_init: fuzz_factor must not be 0\n");
        abort();
    }
    te_fuzz_init_seed = fuzz_seed;
    te_fuzz_init_factor = fuzz_factor;
    __atomic_add_fetch(&te_fuzz_init_gen, 1, __ATOMIC_SEQ_CST);
}

int te_derive_cfg(tcpedit_t *t)
{
    te_dev_cfg_t *c = &t->cfg;
    long v;
    uint32_t seed = 1, rnd = 0;

    te_cfg_defaults(c, t->dlt);
    free(t->portlut);
    t->portlut = NULL;
    t->fuzz_seed = 0;
    t->fuzz_factor = 8;

    /* AutoOpts flags-cant / flags-must (tcpedit_opts.def, en10mb_opts.def) */
    if (conflict(t, OPT_SEED, OPT_FUZZ_SEED) || conflict(t, OPT_PNAT, OPT_SRCIPMAP) ||
        conflict(t, OPT_PNAT, OPT_DSTIPMAP) || conflict(t, OPT_ENET_MAC_SEED, OPT_ENET_SMAC) ||
        conflict(t, OPT_ENET_MAC_SEED, OPT_ENET_DMAC) || conflict(t, OPT_ENET_MAC_SEED, OPT_ENET_SUBSMAC) ||
        requires_(t, OPT_FUZZ_FACTOR, OPT_FUZZ_SEED) || requires_(t, OPT_ENET_VLAN_TAG, OPT_ENET_VLAN) ||
        requires_(t, OPT_ENET_VLAN_CFI, OPT_ENET_VLAN) || requires_(t, OPT_ENET_VLAN_PRI, OPT_ENET_VLAN) ||
        requires_(t, OPT_ENET_MAC_SEED_KEEP_BYTES, OPT_ENET_MAC_SEED))
        return -1;

    if (t->have[OPT_PNAT]) { /* parse_args.c:42-68 */
        c->rewrite_ip = 1;
        if (!parse_cidr_map(t, t->stack[OPT_PNAT][0], c->cidrmap1, &c->n_cidrmap1, "--pnat"))
            return -1;
        if (t->nstack[OPT_PNAT] > 1 &&
            !parse_cidr_map(t, t->stack[OPT_PNAT][1], c->cidrmap2, &c->n_cidrmap2, "--pnat"))
            return -1;
    }
    if (t->have[OPT_SRCIPMAP]) {
        c->rewrite_ip = 1;
        if (!parse_cidr_map(t, t->arg[OPT_SRCIPMAP], c->srcipmap, &c->n_srcipmap, "--srcipmap"))
            return -1;
    }
    if (t->have[OPT_DSTIPMAP]) {
        c->rewrite_ip = 1;
        if (!parse_cidr_map(t, t->arg[OPT_DSTIPMAP], c->dstipmap, &c->n_dstipmap, "--dstipmap"))
            return -1;
    }
    if (c->n_cidrmap1 && !c->n_cidrmap2) { /* :89-94 one -N serves both directions */
        memcpy(c->cidrmap2, c->cidrmap1, sizeof(c->cidrmap1));
        c->n_cidrmap2 = c->n_cidrmap1;
        free(t->cspill[1]);
        t->cspill[1] = NULL;
        if (c->n_cidrmap1 > TE_MAX_CIDRMAP) {
            const size_t nb = sizeof(te_cidrmap_t) * (size_t)(c->n_cidrmap1 - TE_MAX_CIDRMAP);
            t->cspill[1] = malloc(nb);
            if (!t->cspill[1]) {
                te_seterr(t, "out of memory");
                return -1;
            }
            memcpy(t->cspill[1], t->cspill[0], nb);
        }
    }
    c->fixcsum = t->have[OPT_FIXCSUM] != 0;
    c->fixhdrlen = t->have[OPT_FIXHDRLEN] != 0;
    c->efcs = t->have[OPT_EFCS] != 0;
    if (t->have[OPT_TTL]) { /* :109-131 */
        const char *a = t->arg[OPT_TTL];
        c->ttl_mode = strchr(a, '+') ? TE_TTL_ADD : (strchr(a, '-') ? TE_TTL_SUB : TE_TTL_SET);
        long ttl = strtol(a, NULL, 10);
        if (ttl < 0)
            ttl = -ttl;
        if (ttl > 255) {
            te_seterr(t, "Invalid --ttl value (must be 0-255): %ld", ttl);
            return -1;
        }
        c->ttl_value = (uint32_t)ttl;
    }
    if (t->have[OPT_TOS]) {
        if (!num_arg(t, OPT_TOS, 0, 255, &v))
            return -1;
        c->tos = (int32_t)v;
    }
    if (t->have[OPT_TCLASS]) {
        if (!num_arg(t, OPT_TCLASS, 0, 255, &v))
            return -1;
        c->tclass = (int32_t)v;
    }
    if (t->have[OPT_FLOWLABEL]) {
        if (!num_arg(t, OPT_FLOWLABEL, 0, 1048575, &v))
            return -1;
        c->flowlabel = (int32_t)v;
    }
    if (t->have[OPT_MTU]) {
        if (!num_arg(t, OPT_MTU, 1, 262144, &v))
            return -1;
        c->mtu = (int32_t)v;
    }
    c->mtu_truncate = t->have[OPT_MTU_TRUNC] != 0;
    c->skip_broadcast = t->have[OPT_SKIPBROADCAST] != 0;
    if (t->have[OPT_FIXLEN]) {
        const char *a = t->arg[OPT_FIXLEN];
        if (!strcmp(a, "pad"))
            c->fixlen = TE_FIXLEN_PAD;
        else if (!strcmp(a, "trunc"))
            c->fixlen = TE_FIXLEN_TRUNC;
        else if (!strcmp(a, "del"))
            c->fixlen = TE_FIXLEN_DEL;
        else {
            te_seterr(t, "Invalid --fixlen=%s", a);
            return -1;
        }
    }
    if (t->have[OPT_TCP_SEQUENCE]) { /* :180-188 */
        if (!num_arg(t, OPT_TCP_SEQUENCE, 1, 0xffffffffL, &v))
            return -1;
        c->tcp_sequence_enable = 1;
        seed = (uint32_t)v;
        for (int i = 0; i < 5; ++i)
            rnd = te_tcpr_random(&seed);
        c->tcp_sequence_adjust = rnd;
    }
    if (t->have[OPT_PORTMAP]) { /* :191-216 */
        pm_ent_t *ents = NULL;
        int n = 0, cap = 0;
        for (int k = 0; k < t->nstack[OPT_PORTMAP]; k++) {
            if (!pm_parse(t->stack[OPT_PORTMAP][k], &ents, &n, &cap)) {
                te_seterr(t, "Unable to parse --portmap=%s", t->stack[OPT_PORTMAP][k]);
                free(ents);
                return -1;
            }
        }
        /* map_port() returns the first match in list order: build a LUT whose
         * index is the port as loaded from the packet (network order bytes) */
        t->portlut = malloc(65536 * sizeof(uint16_t));
        uint8_t *set = calloc(65536, 1);
        for (int p = 0; p < 65536; p++)
            t->portlut[p] = (uint16_t)p;
        for (int i = 0; i < n; i++) {
            uint16_t f = (uint16_t)ents[i].from;
            if (!set[f]) {
                set[f] = 1;
                t->portlut[f] = (uint16_t)ents[i].to;
            }
        }
        free(set);
        free(ents);
        c->has_portmap = 1;
        pm_sparse(t);
    }
    if (t->have[OPT_SEED]) { /* :218-238 */
        c->rewrite_ip = 1;
        if (!num_arg(t, OPT_SEED, 0x80000000L * -1, 0xffffffffL, &v))
            return -1;
        seed = (uint32_t)v;
    } else if (t->have[OPT_FUZZ_SEED]) {
        if (!num_arg(t, OPT_FUZZ_SEED, 0, 0xffffffffL, &v))
            return -1;
        seed = (uint32_t)v;
        if (t->have[OPT_FUZZ_FACTOR]) {
            if (!num_arg(t, OPT_FUZZ_FACTOR, 1, 0xffffffffL, &v))
                return -1;
            t->fuzz_factor = (uint32_t)v;
        }
    }
    for (int i = 0; i < 5; ++i)
        rnd = te_tcpr_random(&seed);
    if (t->have[OPT_SEED])
        c->seed = seed;
    if (t->have[OPT_FUZZ_SEED]) { /* :232-235; fuzzing_init (tcprewrite.c:102-103) */
        t->fuzz_seed = seed;
        c->fuzz_seed = seed;
        c->fuzz_factor = t->fuzz_factor;
    }
    if (t->have[OPT_ENDPOINTS]) {
        c->rewrite_ip = 1;
        if (!parse_endpoints(t, t->arg[OPT_ENDPOINTS])) {
            if (!t->pub.runtime.errstr[0])
                te_seterr(t, "Unable to parse --endpoints=%s", t->arg[OPT_ENDPOINTS]);
            return -1;
        }
    }

    /* tcpedit_dlt_post_args (dlt_plugins.c:168-204): encoder = --dlt or decoder */
    c->decoder = te_decoder_of(t->dlt);
    if (c->decoder < 0) {
        te_seterr(t, "No DLT plugin available for source DLT: 0x%x (this build: EN10MB, LINUX_SLL, LINUX_SLL2, "
                     "RAW, NULL, LOOP, PPP_SERIAL, C_HDLC, JUNIPER_ETHER, IEEE802_11, IEEE802_11_RADIO)", t->dlt);
        return -1;
    }
    c->encoder = te_default_encoder(c->decoder);
    c->out_linktype = t->dlt;
    if (t->have[OPT_DLT]) { /* tcpedit_dlt_getplugin_byname: the plugins' registered names */
        static const struct {
            const char *name;
            int enc, dlt;
        } plugins[] = {{"enet", TE_ENC_EN10MB, 1},      {"user", TE_ENC_USER, 147},    {"hdlc", TE_ENC_HDLC, 104},
                       {"linuxsll", TE_ENC_NOENC, 113}, {"linuxsll2", TE_ENC_NOENC, 276}, {"raw", TE_ENC_NOENC, 12},
                       {"null", TE_ENC_NOENC, 0},       {"loop", TE_ENC_NOENC, 108},   {"pppserial", TE_ENC_PPP, 50},
                       {"jnpr_eth", TE_ENC_NOENC, 178}, {"ieee80211", TE_ENC_NOENC, 105}, {"radiotap", TE_ENC_NOENC, 127}};
        size_t k = 0;
        while (k < sizeof(plugins) / sizeof(plugins[0]) && strcmp(plugins[k].name, t->arg[OPT_DLT]) != 0)
            k++;
        if (k == sizeof(plugins) / sizeof(plugins[0])) {
            te_seterr(t, "No output DLT plugin available for: %s", t->arg[OPT_DLT]);
            return -1;
        }
        c->encoder = plugins[k].enc;
        c->out_linktype = plugins[k].dlt;
    }
    { /* dlt_user_parse_opts (user.c:158-205): --user-dlt, else the decoder's DLT */
        long v = 1;
        if (t->have[OPT_USER_DLT] && !num_arg(t, OPT_USER_DLT, 0, 65535, &v))
            return -1;
        if (c->encoder == TE_ENC_USER)
            c->out_linktype = t->have[OPT_USER_DLT] ? (int32_t)v : t->dlt;
        for (int k = 0; k < t->nstack[OPT_USER_DLINK]; k++) {
            uint8_t *dst = k == 0 ? c->user_l2server : c->user_l2client;
            const int n = read_hexstring(t->stack[OPT_USER_DLINK][k], dst, 255);
            if (n < 0) {
                te_seterr(t, "Invalid hex string byte in --user-dlink=%s", t->stack[OPT_USER_DLINK][k]);
                return -1;
            }
            if (k == 0) {
                c->user_length = n;
                memcpy(c->user_l2client, c->user_l2server, (size_t)n);
            } else if (n != c->user_length) {
                te_seterr(t, "both --dlink's must contain the same number of bytes");
                return -1;
            }
        }
        if (c->encoder == TE_ENC_USER && c->user_length < 0) {
            te_seterr(t, "--dlt=user requires --user-dlink");
            return -1;
        }
    }
    /* (without --hdlc-address / --hdlc-control dlt_hdlc_encode falls back on the decoded
       extra's first int, hdlc.c:270-288: a tagged Ethernet frame's vlan flag, else a soft
       error written as its memmove left it -- served on the device, edit_pkt.hpp hdlc_encode) */
    { /* dlt_hdlc_parse_opts (hdlc.c:156-180) */
        long v;
        if (t->have[OPT_HDLC_CONTROL]) {
            if (!num_arg(t, OPT_HDLC_CONTROL, 0, 255, &v))
                return -1;
            c->hdlc_control = (uint32_t)v;
        }
        if (t->have[OPT_HDLC_ADDRESS]) {
            if (!num_arg(t, OPT_HDLC_ADDRESS, 0, 255, &v))
                return -1;
            c->hdlc_address = (uint32_t)v;
        }
    }
    c->l2_skip_broadcast = t->have[OPT_SKIPL2BROADCAST] != 0;

    /* dlt_en10mb_parse_opts (en10mb.c:226-396) */
    for (int k = 0; k < t->nstack[OPT_ENET_SUBSMAC]; k++) {
        const char *in = t->stack[OPT_ENET_SUBSMAC][k];
        size_t L = strlen(in), nent = L / 36 + 1; /* SUBSMAC_ENTRY_LEN + 1 */
        for (size_t e = 0; e < nent; e++) {
            size_t off = e * 36;
            if (L - off < 35 || c->n_subs >= TE_MAX_SUBS) {
                te_seterr(t, "Unable to parse --enet-subsmac=%s", in);
                return -1;
            }
            uint8_t *ent = c->subs[c->n_subs];
            memset(ent, 0, 12);
            if (dual_mac(in + off, ent, ent + 6) != 3) {
                te_seterr(t, "Unable to parse --enet-subsmac=%s", in);
                return -1;
            }
            c->n_subs++;
        }
    }
    if (t->have[OPT_ENET_MAC_SEED]) {
        if (!num_arg(t, OPT_ENET_MAC_SEED, 0x80000000L * -1, 0xffffffffL, &v))
            return -1;
        c->random_set = (uint32_t)v;
        uint32_t st = c->random_set;
        for (int i = 0; i < 6; i++) { /* six distinct mask bytes */
            uint8_t m = (uint8_t)te_tcpr_random(&st);
            int dup = 0;
            for (int j = 0; j < i; j++)
                dup |= c->random_mask[j] == m;
            if (dup)
                i--;
            else
                c->random_mask[i] = m;
        }
        c->random_set = st; /* en10mb.c:253-261 leaves the PRNG state in random.set */
        if (t->have[OPT_ENET_MAC_SEED_KEEP_BYTES]) {
            if (!num_arg(t, OPT_ENET_MAC_SEED_KEEP_BYTES, 1, 6, &v))
                return -1;
            c->random_keep = (int32_t)v;
        }
    }
    if (t->have[OPT_ENET_DMAC]) {
        int r = dual_mac(t->arg[OPT_ENET_DMAC], c->intf1_dmac, c->intf2_dmac);
        c->mac_mask |= ((r & 1) ? TE_MASK_DMAC1 : 0) | ((r & 2) ? TE_MASK_DMAC2 : 0);
    }
    if (t->have[OPT_ENET_SMAC]) {
        int r = dual_mac(t->arg[OPT_ENET_SMAC], c->intf1_smac, c->intf2_smac);
        c->mac_mask |= ((r & 1) ? TE_MASK_SMAC1 : 0) | ((r & 2) ? TE_MASK_SMAC2 : 0);
    }
    if (t->have[OPT_ENET_VLAN]) {
        const char *a = t->arg[OPT_ENET_VLAN];
        if (!strcmp(a, "add"))
            c->vlan = TE_VLAN_ADD;
        else if (!strcmp(a, "del"))
            c->vlan = TE_VLAN_DEL;
        else {
            te_seterr(t, "Invalid --enet-vlan=%s", a);
            return -1;
        }
        if (c->vlan == TE_VLAN_ADD) {
            if (!t->have[OPT_ENET_VLAN_TAG]) {
                te_seterr(t, "Must specify a new 802.1 VLAN tag if vlan mode is add");
                return -1;
            }
            if (!num_arg(t, OPT_ENET_VLAN_TAG, 0, 4095, &v))
                return -1;
            c->vlan_tag = (uint32_t)v;
            if (t->have[OPT_ENET_VLAN_PRI]) {
                if (!num_arg(t, OPT_ENET_VLAN_PRI, 0, 7, &v))
                    return -1;
                c->vlan_pri = (uint32_t)v;
            }
            if (t->have[OPT_ENET_VLAN_CFI]) {
                if (!num_arg(t, OPT_ENET_VLAN_CFI, 0, 1, &v))
                    return -1;
                c->vlan_cfi = (uint32_t)v;
            }
        }
        if (t->have[OPT_ENET_VLAN_PROTO]) {
            const char *p = t->arg[OPT_ENET_VLAN_PROTO];
            if (!strcasecmp(p, "802.1q"))
                c->vlan_proto = 0x8100;
            else if (!strcasecmp(p, "802.1ad"))
                c->vlan_proto = 0x88A8;
            else {
                te_seterr(t, "VLAN protocol \"%s\" is invalid", p);
                return -1;
            }
        }
    }
    c->skip_soft_errors = t->have[OPT_SKIP_SOFT_ERRORS] != 0;
    if (te_check_decoder_cfg(t, 0) < 0)
        return -1;
    t->post_args_done = 1;
    t->dev_dirty = 1;
    t->fz_seeded = 0; /* fuzzing_init (tcprewrite.c:103) follows post_args */
    te_sync_pub(t);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* programmatic setters (tcpedit_api.c:33-353)                               */
/* ------------------------------------------------------------------------- */
static int setter_done(tcpedit_t *t)
{
    t->opt_src |= TE_SRC_SETTERS;
    t->dev_dirty = 1;
    te_sync_pub(t);
    return TCPEDIT_OK;
}

#define SETFLAG(fn, field)                     \
    int fn(tcpedit_t *t, bool v)               \
    {                                          \
        if (!t)                                \
            return TCPEDIT_ERROR;              \
        t->cfg.field = v ? 1 : 0;              \
        return setter_done(t);                 \
    }
SETFLAG(tcpedit_set_skip_broadcast, skip_broadcast)
SETFLAG(tcpedit_set_fixcsum, fixcsum)
SETFLAG(tcpedit_set_fixhdrlen, fixhdrlen)
SETFLAG(tcpedit_set_efcs, efcs)
SETFLAG(tcpedit_set_mtu_truncate, mtu_truncate)

int tcpedit_set_ttl_mode(tcpedit_t *t, tcpedit_ttl_mode m)
{
    if (!t || m < TCPEDIT_TTL_MODE_OFF || m > TCPEDIT_TTL_MODE_SUB)
        return TCPEDIT_ERROR;
    t->cfg.ttl_mode = m;
    return setter_done(t);
}
int tcpedit_set_ttl_value(tcpedit_t *t, uint8_t v)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.ttl_value = v;
    return setter_done(t);
}
int tcpedit_set_tos(tcpedit_t *t, uint8_t v)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.tos = v;
    return setter_done(t);
}
int tcpedit_set_tclass(tcpedit_t *t, uint8_t v)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.tclass = v;
    return setter_done(t);
}
int tcpedit_set_flowlabel(tcpedit_t *t, uint32_t v)
{
    if (!t || v > 1048575)
        return TCPEDIT_ERROR;
    t->cfg.flowlabel = (int32_t)v;
    return setter_done(t);
}
int tcpedit_set_seed(tcpedit_t *t)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.seed = (uint32_t)random();
    t->cfg.rewrite_ip = 1;
    return setter_done(t);
}
int tcpedit_set_mtu(tcpedit_t *t, int mtu)
{
    if (!t || mtu < 1 || mtu > 262144)
        return TCPEDIT_ERROR;
    t->cfg.mtu = mtu;
    return setter_done(t);
}
int tcpedit_set_maxpacket(tcpedit_t *t, int v)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->pub.maxpacket = v; /* tcpedit_api.c:257-262: stored, never read on the edit path */
    return TCPEDIT_OK;
}
int tcpedit_set_fixlen(tcpedit_t *t, tcpedit_fixlen v)
{
    if (!t || v < TCPEDIT_FIXLEN_OFF || v > TCPEDIT_FIXLEN_DEL)
        return TCPEDIT_ERROR;
    t->cfg.fixlen = v;
    return setter_done(t);
}
int tcpedit_set_tcp_sequence(tcpedit_t *t, uint32_t adjust)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.tcp_sequence_enable = 1;
    t->cfg.tcp_sequence_adjust = adjust;
    return setter_done(t);
}
int tcpedit_set_cidrmap_s2c(tcpedit_t *t, char *s)
{
    if (!t || !s || !parse_cidr_map(t, s, t->cfg.cidrmap2, &t->cfg.n_cidrmap2, "cidrmap"))
        return TCPEDIT_ERROR;
    t->cfg.rewrite_ip = 1;
    return setter_done(t);
}
int tcpedit_set_cidrmap_c2s(tcpedit_t *t, char *s)
{
    if (!t || !s || !parse_cidr_map(t, s, t->cfg.cidrmap1, &t->cfg.n_cidrmap1, "cidrmap"))
        return TCPEDIT_ERROR;
    t->cfg.rewrite_ip = 1;
    return setter_done(t);
}
int tcpedit_set_srcip_map(tcpedit_t *t, char *s)
{
    if (!t || !s || !parse_cidr_map(t, s, t->cfg.srcipmap, &t->cfg.n_srcipmap, "srcipmap"))
        return TCPEDIT_ERROR;
    t->cfg.rewrite_ip = 1;
    return setter_done(t);
}
int tcpedit_set_dstip_map(tcpedit_t *t, char *s)
{
    if (!t || !s || !parse_cidr_map(t, s, t->cfg.dstipmap, &t->cfg.n_dstipmap, "dstipmap"))
        return TCPEDIT_ERROR;
    t->cfg.rewrite_ip = 1;
    return setter_done(t);
}
int tcpedit_set_port_map(tcpedit_t *t, char *s)
{
    pm_ent_t *ents = NULL;
    int n = 0, cap = 0;
    if (!t || !s || !pm_parse(s, &ents, &n, &cap)) {
        free(ents);
        return TCPEDIT_ERROR;
    }
    if (!t->portlut) {
        t->portlut = malloc(65536 * sizeof(uint16_t));
        for (int p = 0; p < 65536; p++)
            t->portlut[p] = (uint16_t)p;
    }
    /* appended records only apply to ports no earlier record matched */
    uint8_t *set = calloc(65536, 1);
    for (int p = 0; p < 65536; p++)
        set[p] = t->portlut[p] != p;
    for (int i = 0; i < n; i++) {
        uint16_t f = (uint16_t)ents[i].from;
        if (!set[f]) {
            set[f] = 1;
            t->portlut[f] = (uint16_t)ents[i].to;
        }
    }
    free(set);
    free(ents);
    t->cfg.has_portmap = 1;
    pm_sparse(t);
    return setter_done(t);
}

/* tcpedit_set_encoder_dltplugin_byid/_byname (tcpedit_api.c:33-104): select the encoder
 * once; the plugins this build carries are enet (DLT_EN10MB), user (DLT_USER0) and hdlc
 * (DLT_C_HDLC) */
static int set_encoder(tcpedit_t *t, int enc)
{
    static const char *names[] = {"enet", "user", "hdlc"};
    if (t->encoder_set) {
        te_seterr(t, "You have already selected a DLT encoder: %s", names[t->cfg.encoder]);
        return TCPEDIT_ERROR;
    }
    t->encoder_set = 1;
    t->cfg.encoder = enc;
    t->cfg.out_linktype = enc == TE_ENC_HDLC ? 104 : enc == TE_ENC_USER ? t->dlt : 1;
    return setter_done(t);
}
int tcpedit_set_encoder_dltplugin_byid(tcpedit_t *t, int dlt)
{
    if (!t)
        return TCPEDIT_ERROR;
    const int enc = dlt == 1 ? TE_ENC_EN10MB : dlt == 147 ? TE_ENC_USER : dlt == 104 ? TE_ENC_HDLC : -1;
    if (enc < 0) {
        te_seterr(t, "No output DLT plugin decoder with DLT type: 0x%04x", dlt);
        return TCPEDIT_ERROR;
    }
    return set_encoder(t, enc);
}
int tcpedit_set_encoder_dltplugin_byname(tcpedit_t *t, const char *name)
{
    if (!t || !name)
        return TCPEDIT_ERROR;
    const int enc = !strcmp(name, "enet") ? TE_ENC_EN10MB
                    : !strcmp(name, "user") ? TE_ENC_USER
                    : !strcmp(name, "hdlc") ? TE_ENC_HDLC : -1;
    if (enc < 0) {
        te_seterr(t, "No output DLT plugin available for: %s", name);
        return TCPEDIT_ERROR;
    }
    return set_encoder(t, enc);
}

/* EN10MB plugin setters (plugins/dlt_en10mb/en10mb_api.c:38-192): they write the
 * plugin config directly; set_mac adds the mask bit with `+=` as the reference does */
int tcpedit_en10mb_set_mac(tcpedit_t *t, char *mac, tcpedit_mac_mask mask)
{
    if (!t || !mac)
        return TCPEDIT_ERROR;
    uint8_t a[6] = {0, 0, 0, 0, 0, 0};
    mac_from_str(mac, a);
    te_dev_cfg_t *c = &t->cfg;
    switch (mask) {
    case TCPEDIT_MAC_MASK_DMAC1: memcpy(c->intf1_dmac, a, 6); break;
    case TCPEDIT_MAC_MASK_DMAC2: memcpy(c->intf2_dmac, a, 6); break;
    case TCPEDIT_MAC_MASK_SMAC1: memcpy(c->intf1_smac, a, 6); break;
    case TCPEDIT_MAC_MASK_SMAC2: memcpy(c->intf2_smac, a, 6); break;
    default: return TCPEDIT_OK; /* the reference's switch has no other case */
    }
    c->mac_mask += (int32_t)mask;
    return setter_done(t);
}
int tcpedit_en10mb_set_vlan_mode(tcpedit_t *t, tcpedit_vlan vlan)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.vlan = (int32_t)vlan;
    return setter_done(t);
}
int tcpedit_en10mb_set_vlan_tag(tcpedit_t *t, uint16_t tag)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.vlan_tag = tag;
    return setter_done(t);
}
int tcpedit_en10mb_set_vlan_priority(tcpedit_t *t, uint8_t priority)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.vlan_pri = priority;
    return setter_done(t);
}
int tcpedit_en10mb_set_vlan_cfi(tcpedit_t *t, uint8_t cfi)
{
    if (!t)
        return TCPEDIT_ERROR;
    t->cfg.vlan_cfi = cfi;
    return setter_done(t);
}

/* one CIDR (cidr2cidr, cidr.c:130-221) for tcpprep's option parser (tp_api.c) */
int te_parse_cidr(char *s, te_cidr_t *c) { return parse_one_cidr(s, c); }
