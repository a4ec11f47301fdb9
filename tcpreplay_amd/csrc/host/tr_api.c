/*
 * tr_api.c -- tcpreplay's replay passes with --unique-ip on the GPU (include/tcpreplay_hip.h).
 *
 * The host side of send_packets (src/send_packets.c:379-646) for file output: the record
 * walk libpcap's reader makes (a record past MAX_SNAPLEN or past the end stops it), the
 * pass loop with increment_iteration (:362-372) deciding which passes edit, and the
 * pcap_dump header (sendpacket.c:945-968: pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN)).
 * safe_pcap_next's rules (src/common/utils.c:131-169) hold on the walk: a zero len or
 * caplen (or len > MAX_SNAPLEN) ends the run after the first pass's earlier records, and
 * the kernels trim caplen to len.  Each
 * pass runs on the device (tcpreplay_kernels.hip) and lands in one device output buffer.
 */
#include <hip/hip_runtime_api.h>
#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/tcpreplay_hip.h"
#include "tcpreplay_hip_dev.h"

struct tcpreplay_hip_s {
    uint32_t loops;
    int unique_ip, preload;
    double unique_loops;
    tr_list_t list;     /* --include / --exclude (n = 0: none) */
    int reader_exit;    /* the last replay ended at safe_pcap_next's exit */
    int64_t out_len;    /* the bytes the last replay wrote */
    char err[512];
};

int tcpreplay_hip_reader_exited(tcpreplay_hip_t *t) { return t ? t->reader_exit : 0; }
int64_t tcpreplay_hip_output_len(tcpreplay_hip_t *t) { return t ? t->out_len : 0; }

/* parse_list (src/common/list.c:61-130): ',' tokens (strtok_r drops empty ones), each
   "^[0-9]+(-([0-9]+|\s*))?$"; add_to_list (:36-50) takes min by strtoull(.., 0), max = min
   without a '-', 0 for an open "N-" */
int tr_list_parse(tr_list_t *l, const char *arg, int exclude, char *err, size_t errlen)
{
    tr_list_free(l);
    l->exclude = exclude;
    char *buf = arg ? strdup(arg) : NULL;
    uint32_t cap = 0;
    int ok = buf != NULL;
    char *tok = NULL;
    for (char *e = ok ? strtok_r(buf, ",", &tok) : NULL; e && ok; e = strtok_r(NULL, ",", &tok)) {
        char *p = e, *second = NULL;
        ok = isdigit((unsigned char)*p) != 0;
        while (isdigit((unsigned char)*p))
            p++;
        if (ok && *p == '-') {
            *p++ = 0;
            second = p;
            if (isdigit((unsigned char)*p))
                while (isdigit((unsigned char)*p))
                    p++;
            else
                while (isspace((unsigned char)*p))
                    p++;
        }
        ok = ok && !*p;
        if (ok && l->n == cap) {
            cap = cap ? 2 * cap : 16;
            uint64_t *g = realloc(l->rng, 2 * sizeof(uint64_t) * cap);
            ok = g != NULL;
            if (g)
                l->rng = g;
        }
        if (ok) {
            l->rng[2 * l->n] = strtoull(e, NULL, 0);
            l->rng[2 * l->n + 1] = second ? (second[0] ? strtoull(second, NULL, 0) : 0) : l->rng[2 * l->n];
            l->n++;
        }
    }
    free(buf);
    if (!ok || !l->n) {
        snprintf(err, errlen, "Unable to parse include/exclude rule: %s", arg ? arg : "(null)");
        tr_list_free(l);
        return -1;
    }
    return 0;
}

void tr_list_free(tr_list_t *l)
{
    free(l->rng);
    l->rng = NULL;
    l->n = 0;
}

static int tr_err(tcpreplay_hip_t *t, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t->err, sizeof t->err, fmt, ap);
    va_end(ap);
    return -1;
}

tcpreplay_hip_t *tcpreplay_hip_init(void)
{
    tcpreplay_hip_t *t = calloc(1, sizeof *t);
    if (t) {
        t->loops = 1;           /* tcpreplay_opts.def: --loop default 1 */
        t->unique_loops = 1.0;  /* tcpreplay_api.c:108 */
    }
    return t;
}

void tcpreplay_hip_close(tcpreplay_hip_t *t)
{
    if (t)
        tr_list_free(&t->list);
    free(t);
}

const char *tcpreplay_hip_geterr(tcpreplay_hip_t *t) { return t ? t->err : "no context"; }

int tcpreplay_hip_set_loop(tcpreplay_hip_t *t, uint32_t v)
{
    if (!t)
        return -1;
    if (v == 0) /* --loop=0 loops forever: no file output ends */
        return tr_err(t, "--loop=0 (forever) has no end to write");
    t->loops = v;
    return 0;
}

int tcpreplay_hip_set_unique_ip(tcpreplay_hip_t *t, bool v)
{
    if (!t)
        return -1;
    t->unique_ip = v;
    return 0;
}

int tcpreplay_hip_set_unique_ip_loops(tcpreplay_hip_t *t, int v)
{
    if (!t)
        return -1;
    if (v < 1) /* tcpreplay_api.c:286-288 */
        return tr_err(t, "--unique-ip-loops requires loop count >= 1.0");
    t->unique_loops = v;
    return 0;
}

int tcpreplay_hip_set_preload_pcap(tcpreplay_hip_t *t, bool v)
{
    if (!t)
        return -1;
    t->preload = v;
    return 0;
}

int tcpreplay_hip_parse_args(tcpreplay_hip_t *t, int argc, char **argv)
{
    if (!t)
        return -1;
    int uloops_seen = 0;
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i], *eq = strchr(a, '=');
        const size_t nl = eq ? (size_t)(eq - a) : strlen(a);
        const char *v = eq ? eq + 1 : NULL;
#define OPT(n) (nl == sizeof(n) - 1 && !strncmp(a, n, nl))
        if (OPT("--loop")) {
            if (!v || tcpreplay_hip_set_loop(t, (uint32_t)strtoul(v, NULL, 0)) < 0)
                return v ? -1 : tr_err(t, "--loop needs a value");
        } else if (OPT("--unique-ip")) {
            t->unique_ip = 1;
        } else if (OPT("--unique-ip-loops")) {
            if (!v)
                return tr_err(t, "--unique-ip-loops needs a value");
            t->unique_loops = atof(v); /* tcpreplay_api.c:285 */
            if (t->unique_loops < 1.0)
                return tr_err(t, "--unique-ip-loops requires loop count >= 1.0");
            uloops_seen = 1;
        } else if (OPT("--preload-pcap") || OPT("-K")) {
            t->preload = 1;
        } else if (OPT("--include") || OPT("--exclude")) {
            /* tcpreplay_opts.def:305-360 (max 1, flags-cant each other) */
            if (!v)
                return tr_err(t, "%.*s needs a value", (int)nl, a);
            if (t->list.n)
                return tr_err(t, "--include and --exclude: one packet list at most");
            if (tr_list_parse(&t->list, v, a[2] == 'e', t->err, sizeof t->err) < 0)
                return -1;
        } else {
            return tr_err(t, "unknown or unserved tcpreplay option %s", a);
        }
#undef OPT
    }
    if (uloops_seen && !t->unique_ip) /* tcpreplay_opts.def:585: flags-must unique-ip */
        return tr_err(t, "--unique-ip-loops requires --unique-ip");
    return 0;
}

size_t tcpreplay_hip_output_bound(tcpreplay_hip_t *t, size_t len)
{
    const size_t body = len > 24 ? len - 24 : 0;
    return 24 + (size_t)(t ? t->loops : 1) * body;
}

static uint32_t rd32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            tr_err(t, "%s: %s", #x, hipGetErrorString(e_));                       \
            goto fail;                                                            \
        }                                                                         \
    } while (0)

int64_t tcpreplay_hip_replay_to_pcap(tcpreplay_hip_t *t, const uint8_t *pcap, size_t len, uint8_t *out, size_t cap,
                                     uint64_t *failed)
{
    if (!t || !pcap || !out || !failed)
        return -1;
    if (len < 24)
        return tr_err(t, "pcap image too short");
    uint32_t magic;
    memcpy(&magic, pcap, 4);
    int sw, nsec;
    switch (magic) {
    case 0xa1b2c3d4u: sw = 0; nsec = 0; break;
    case 0xd4c3b2a1u: sw = 1; nsec = 0; break;
    case 0xa1b23c4du: sw = 0; nsec = 1; break;
    case 0x4d3cb2a1u: sw = 1; nsec = 1; break;
    default: return tr_err(t, "not a pcap file (magic 0x%08x)", magic);
    }
    if ((rd32(pcap + 20, sw) & 0x03ffffffu) != 1 && t->unique_ip)
        return tr_err(t, "--unique-ip is served for DLT_EN10MB captures only");
    if (cap < tcpreplay_hip_output_bound(t, len))
        return tr_err(t, "output buffer smaller than tcpreplay_hip_output_bound");
    t->reader_exit = 0;
    t->out_len = 0;
    /* libpcap's walk: a record past MAX_SNAPLEN or past the end stops the read; then
       safe_pcap_next (send_packets.c:955,985 -> src/common/utils.c:131-169): a len past
       MAX_SNAPLEN or a zero len or caplen exit(-1)s in the first pass, after the records
       before it were sent (the kernels trim len < caplen) */
    uint64_t n = 0, ncap = 1024;
    uint64_t *off = malloc(ncap * sizeof *off);
    int reader_exit = 0;
    for (size_t o = 24; off && o + 16 <= len;) {
        const uint32_t cl = rd32(pcap + o + 8, sw), pl = rd32(pcap + o + 12, sw);
        if (cl > 262144u || o + 16 + cl > len)
            break;
        if (pl > 262144u || !pl || !cl) {
            reader_exit = 1;
            break;
        }
        if (n == ncap) {
            uint64_t *g = realloc(off, 2 * ncap * sizeof *off);
            if (!g) {
                free(off);
                off = NULL;
                break;
            }
            off = g;
            ncap *= 2;
        }
        off[n++] = o;
        o += 16 + cl;
    }
    if (!off)
        return tr_err(t, "out of host memory (record index)");
    uint8_t *d_img = NULL, *d_cache = NULL, *d_out = NULL;
    uint64_t *d_off = NULL, *d_size = NULL, *d_pos = NULL, *d_list = NULL;
    uint64_t *d_nfail = NULL;
    void *d_patch = NULL, *d_temp = NULL, *d_tot = NULL;
    hipStream_t st = NULL;
    int64_t rc = -1;
    const size_t bound = tcpreplay_hip_output_bound(t, len), temp = tr_scan_temp_bytes(n ? n : 1);
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CHK(hipMalloc((void **)&d_img, len));
    CHK(hipMalloc((void **)&d_out, bound));
    CHK(hipMalloc((void **)&d_off, (n ? n : 1) * 8));
    CHK(hipMalloc((void **)&d_size, (n ? n : 1) * 8));
    CHK(hipMalloc((void **)&d_pos, (n ? n : 1) * 8));
    CHK(hipMalloc(&d_patch, (n ? n : 1) * 16));
    CHK(hipMalloc(&d_temp, temp ? temp : 16));
    if (t->preload)
        CHK(hipMalloc((void **)&d_cache, len));
    CHK(hipMalloc((void **)&d_nfail, 8));
    CHK(hipMemsetAsync(d_nfail, 0, 8, st));
    if (t->list.n) {
        CHK(hipMalloc((void **)&d_list, 16 * (size_t)t->list.n));
        CHK(hipMemcpyAsync(d_list, t->list.rng, 16 * (size_t)t->list.n, hipMemcpyHostToDevice, st));
    }
    CHK(hipMemcpyAsync(d_img, pcap, len, hipMemcpyHostToDevice, st));
    if (d_cache)
        CHK(hipMemcpyAsync(d_cache, pcap, len, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(d_off, off, n * 8, hipMemcpyHostToDevice, st));
    {
        static const uint8_t hdr[24] = {0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                        0, 0, 4, 0, 1, 0, 0, 0};
        memcpy(out, hdr, 24);
    }
    uint64_t o = 24, iteration = 0, uniq = 0, last_uniq = 0, fails = 0;
    for (uint32_t pass = 0; pass < (reader_exit ? 1u : t->loops) && n; pass++) {
        TrPass p;
        memset(&p, 0, sizeof p);
        p.img = d_img;
        p.cache = d_cache;
        p.cached = d_cache != NULL;
        p.list = d_list;
        p.nlist = t->list.n;
        p.exclude = t->list.exclude;
        p.nfail = d_nfail;
        p.off = d_off;
        p.n = n;
        p.swapped = sw;
        p.nsec = nsec;
        p.edit = t->unique_ip && uniq && uniq > last_uniq; /* send_packets.c:477 */
        p.iteration = uniq ? uniq - 1 : 0;
        p.size = d_size;
        p.pos = d_pos;
        p.patch = d_patch;
        p.out = d_out + o;
        if (tr_launch_pass(&p, d_temp, temp, st) != 0) {
            tr_err(t, "replay pass launch failed: %s", hipGetErrorString(hipGetLastError()));
            goto fail;
        }
        uint64_t last[2];
        CHK(hipMemcpyAsync(&last[0], d_pos + n - 1, 8, hipMemcpyDeviceToHost, st));
        CHK(hipMemcpyAsync(&last[1], d_size + n - 1, 8, hipMemcpyDeviceToHost, st));
        CHK(hipStreamSynchronize(st));
        const uint64_t pass_bytes = last[0] + last[1];
        o += pass_bytes;
        /* increment_iteration (send_packets.c:362-372) */
        last_uniq = uniq;
        ++iteration;
        if (t->unique_ip)
            uniq = (iteration * 1000) / (uint64_t)(t->unique_loops * 1000.0) + 1;
    }
    CHK(hipMemcpyAsync(out + 24, d_out + 24, o - 24, hipMemcpyDeviceToHost, st));
    {
        uint64_t nf = 0; /* the records whose unique-ip edit failed, over every pass */
        CHK(hipMemcpyAsync(&nf, d_nfail, 8, hipMemcpyDeviceToHost, st));
        CHK(hipStreamSynchronize(st));
        fails = nf;
    }
    *failed = fails;
    t->out_len = (int64_t)o;
    rc = (int64_t)o;
    if (reader_exit) { /* the output holds the first pass's records before it: a return no
                          caller can take for a whole run (tcpreplay exit(-1)s there) */
        t->reader_exit = 1;
        tr_err(t, "safe_pcap_next ERROR: Invalid packet length: packet %llu", (unsigned long long)(n + 1));
        rc = TCPREPLAY_HIP_READER_EXIT;
    }
fail:
    hipFree(d_img);
    hipFree(d_cache);
    hipFree(d_out);
    hipFree(d_off);
    hipFree(d_size);
    hipFree(d_pos);
    hipFree(d_patch);
    hipFree(d_temp);
    hipFree(d_tot);
    hipFree(d_list);
    hipFree(d_nfail);
    if (st)
        hipStreamDestroy(st);
    free(off);
    return rc;
}
