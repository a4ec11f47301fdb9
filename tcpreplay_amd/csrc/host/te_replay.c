/*
 * te_replay.c -- tcpreplay-edit's send loop, batched (include/tcpedit.h tcpedit_replay_*).
 *
 * tcpreplay-edit edits every packet just before it sends it (src/send_packets.c:469-474,
 * tcpedit_packet with intf1's direction) -- one call per packet per --loop pass.  Here a
 * pass is one device batch over the whole capture:
 *   - without --preload-pcap every pass reads the file again (get_next_packet :985): the
 *     pass edits the capture as read;
 *   - with --preload-pcap (-K) the first pass edits libpcap's buffer while caching an
 *     unedited copy of every record (:955-980: caplen + PACKET_HEADROOM bytes, and its
 *     header), and every later pass edits the cached bytes IN PLACE with a copy of the
 *     cached header (:934-950).  So the edits compound from pass to pass: pass
 *     p + 1 edits the first caplen bytes of what pass p left in the cache buffer -- the
 *     edited bytes, and past the edited length the bytes the edit did not touch.
 * The cache lives on the host in the capture's own layout (the cached headers are the
 * file's), and goes up before each cached pass; the device index of the capture serves
 * every pass.  Output: the records as sent, in the -w dump's form (sendpacket.c:485-486
 * pcap_dump into pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN); the timestamp fraction as
 * libpcap's nanosecond read leaves it).
 * The rest of send_packets' per-record steps ride in the same pass (tcpedit_replay_parse_args):
 *   - --include / --exclude (:440-447): a record the list leaves out is read (and cached
 *     under -K) but neither edited nor sent -- on the device the list becomes the batch's
 *     direction array, NOSEND for those records (tr_list_dirbits), so the edit kernels leave
 *     them as read (no RNG draw under --fuzz-seed, the stale-buffer replay sees them read);
 *   - --unique-ip (:477-483): fast_edit_packet on each edited record of the passes where
 *     unique_iteration advanced, on the device over the batch's output (tr_mark: the two
 *     new addresses per record, or a failure: counted, not sent); under -K it lands in the
 *     cache as well (the reference edits the cached bytes in place).
 * Not served (refused): stale static-buffer reads
 *  on a cached pass (the reference reads its cache buffer's headroom there),
 * --fuzz-seed with -K over several passes, non-Ethernet captures (tcpreplay-edit decodes
 * with the interface's DLT, DLT_EN10MB for the dump).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/tcpedit.h"
#include "tcpreplay_hip_dev.h"
#include "te_dev_cfg.h"
#include "te_internal.h"

struct tcpedit_replay_s {
    tcpedit_batch_t *b;
    uint8_t *img;     /* the capture (host copy) */
    uint8_t *cache;   /* -K: the cached records, same layout as img */
    size_t len;
    uint64_t nrec, pass;
    int preload, swapped, nsec;
    /* tcpreplay's per-record steps around the edit */
    tr_list_t list;       /* --include / --exclude (n = 0: none) */
    int list_set;         /* the list is the batch's direction array */
    int unique_ip;
    double unique_loops;
    uint64_t iteration, uniq, last_uniq, failed; /* increment_iteration (send_packets.c:362-372) */
    /* device scratch of the unique-ip step */
    uint64_t *d_off, *d_size, *d_nfail;
    void *d_patch;
    uint64_t cap;
};

static uint32_t rp32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

tcpedit_replay_t *tcpedit_replay_open(tcpedit_t *t, const void *pcap, size_t len, int preload)
{
    if (!t || !pcap || len < 24) {
        if (t)
            te_seterr(t, "tcpedit_replay_open: no capture");
        return NULL;
    }
    tcpedit_replay_t *r = calloc(1, sizeof(*r));
    if (!r)
        return NULL;
    uint32_t magic;
    memcpy(&magic, pcap, 4);
    r->swapped = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    r->nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    r->preload = preload;
    r->unique_loops = 1.0; /* tcpreplay_api.c:108 */
    r->len = len;
    r->img = malloc(len);
    if (!r->img)
        goto fail;
    memcpy(r->img, pcap, len);
    for (size_t p = 24; p + 16 <= len; r->nrec++) { /* libpcap's walk */
        const uint32_t cl = rp32(r->img + p + 8, r->swapped), pl = rp32(r->img + p + 12, r->swapped);
        if (cl > 262144u || p + 16 + cl > len)
            break;
        /* safe_pcap_next (send_packets.c:955,985 -> src/common/utils.c:136-156) exits at
           this record: the batch stops there too (its first pass then fails after the
           records before it were sent) */
        if (pl > 262144u || !pl || !cl)
            break;
        p += 16 + cl;
    }
    if (preload) {
        r->cache = malloc(len);
        if (!r->cache)
            goto fail;
        memcpy(r->cache, pcap, len);
    }
    if (t->cfg.skip_soft_errors) { /* a tcprewrite option: tcpreplay-edit sends every record */
        te_seterr(t, "tcpedit_replay: --skip-soft-errors is tcprewrite's option (tcpreplay-edit drops no record)");
        goto fail;
    }
    if (preload && ((const tcpedit_ref_t *)t)->fuzz_seed) {
        te_seterr(t, "tcpedit_replay: --fuzz-seed with --preload-pcap is not served (its writes past a record "
                     "land in the cache buffer's headroom)");
        goto fail;
    }
    r->b = tcpedit_batch_open(t, r->img, len, NULL, 0, 0);
    if (!r->b)
        goto fail;
    return r;
fail:
    tcpedit_replay_close(r);
    return NULL;
}

void tcpedit_replay_close(tcpedit_replay_t *r)
{
    if (!r)
        return;
    tr_list_free(&r->list);
    hipFree(r->d_off);
    hipFree(r->d_size);
    hipFree(r->d_nfail);
    hipFree(r->d_patch);
    tcpedit_batch_close(r->b);
    free(r->img);
    free(r->cache);
    free(r);
}

/* tcpreplay's options around the edit (tcpreplay_opts.def): --include=LIST / --exclude=LIST
   (:305-360, one of them), --unique-ip (:567-580), --unique-ip-loops=N (:581-595, >= 1,
   needs --unique-ip); before the first pass */
int tcpedit_replay_parse_args(tcpedit_t *t, tcpedit_replay_t *r, int argc, char **argv)
{
    if (!t || !r || argc < 0 || (argc && !argv))
        return TCPEDIT_ERROR;
    if (r->pass) {
        te_seterr(t, "tcpedit_replay_parse_args: after the first pass");
        return TCPEDIT_ERROR;
    }
    int uloops = 0;
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i];
        if (!strncmp(a, "--include=", 10) || !strncmp(a, "--exclude=", 10)) {
            char err[256];
            if (r->list.n) {
                te_seterr(t, "--include and --exclude: one packet list at most");
                return TCPEDIT_ERROR;
            }
            if (tr_list_parse(&r->list, a + 10, a[2] == 'e', err, sizeof err) < 0) {
                te_seterr(t, "%s", err);
                return TCPEDIT_ERROR;
            }
        } else if (!strcmp(a, "--unique-ip")) {
            r->unique_ip = 1;
        } else if (!strncmp(a, "--unique-ip-loops=", 18)) {
            r->unique_loops = atof(a + 18); /* tcpreplay_api.c:285-288 */
            uloops = 1;
            if (r->unique_loops < 1.0) {
                te_seterr(t, "--unique-ip-loops requires loop count >= 1.0");
                return TCPEDIT_ERROR;
            }
        } else {
            te_seterr(t, "tcpedit_replay_parse_args: unknown or unserved tcpreplay option %s", a);
            return TCPEDIT_ERROR;
        }
    }
    if (uloops && !r->unique_ip) {
        te_seterr(t, "--unique-ip-loops requires --unique-ip");
        return TCPEDIT_ERROR;
    }
    return TCPEDIT_OK;
}

uint64_t tcpedit_replay_failed(tcpedit_replay_t *r) { return r ? r->failed : 0; }

/* the list as the batch's direction array, built on the device once (it is the same every
   pass: packet numbers restart at 1, send_packets.c:385,437) */
static int replay_set_list(tcpedit_t *t, tcpedit_replay_t *r)
{
    uint64_t *d_list = NULL;
    uint8_t *d_bits = NULL;
    const uint64_t nb = (r->nrec + 3) / 4;
    if (hipMalloc((void **)&d_list, 16 * (size_t)r->list.n) != hipSuccess ||
        hipMalloc((void **)&d_bits, nb + 16) != hipSuccess ||
        hipMemcpyAsync(d_list, r->list.rng, 16 * (size_t)r->list.n, hipMemcpyHostToDevice, t->stream) != hipSuccess ||
        tr_list_dirbits(d_list, r->list.n, r->list.exclude, r->nrec, d_bits, t->stream) != 0 ||
        hipStreamSynchronize(t->stream) != hipSuccess) {
        hipFree(d_list);
        hipFree(d_bits);
        te_seterr(t, "tcpedit_replay: the packet list's device array: %s", hipGetErrorString(hipGetLastError()));
        return -1;
    }
    hipFree(d_list);
    te_batch_set_dirbits_dev(r->b, d_bits, nb);
    r->list_set = 1;
    return 0;
}

/* fast_edit_packet (send_packets.c:124-257) for the k records of the batch output at
   offs[] on the device: sizes (0: the edit failed) and the {at_s, src, at_d, dst} patches */
static int replay_unique(tcpedit_t *t, tcpedit_replay_t *r, const uint64_t *offs, uint64_t k, uint64_t *size,
                         uint32_t *patch)
{
    if (k > r->cap) {
        hipFree(r->d_off);
        hipFree(r->d_size);
        hipFree(r->d_patch);
        r->d_off = r->d_size = NULL;
        r->d_patch = NULL;
        r->cap = 0;
        if (hipMalloc((void **)&r->d_off, 8 * k) != hipSuccess || hipMalloc((void **)&r->d_size, 8 * k) != hipSuccess ||
            hipMalloc(&r->d_patch, 16 * k) != hipSuccess)
            goto fail;
        r->cap = k;
    }
    if (!r->d_nfail && hipMalloc((void **)&r->d_nfail, 8) != hipSuccess)
        goto fail;
    TrPass p;
    memset(&p, 0, sizeof p);
    p.img = (const uint8_t *)tcpedit_batch_device_output(r->b);
    p.cached = r->preload && r->pass > 0; /* file_cache[idx].cached after the first pass */
    p.off = r->d_off;
    p.n = k;
    p.edit = 1;
    p.iteration = r->uniq - 1;
    p.size = r->d_size;
    p.patch = r->d_patch;
    p.mark_only = 1;
    if (hipMemcpyAsync(r->d_off, offs, 8 * k, hipMemcpyHostToDevice, t->stream) != hipSuccess ||
        tr_launch_pass(&p, NULL, 0, t->stream) != 0 ||
        hipMemcpyAsync(size, r->d_size, 8 * k, hipMemcpyDeviceToHost, t->stream) != hipSuccess ||
        hipMemcpyAsync(patch, r->d_patch, 16 * k, hipMemcpyDeviceToHost, t->stream) != hipSuccess ||
        hipStreamSynchronize(t->stream) != hipSuccess)
        goto fail;
    return 0;
fail:
    te_seterr(t, "tcpedit_replay: the unique-ip step on the device: %s", hipGetErrorString(hipGetLastError()));
    return -1;
}

static void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

/* bytes one pass can write: every record grows by at most its slot's room */
size_t tcpedit_replay_bound(tcpedit_t *t, tcpedit_replay_t *r)
{
    return r ? tcpedit_output_bound(t, r->img, r->len) - 24 + 16 * r->nrec : 0;
}

int tcpedit_replay_pass(tcpedit_t *t, tcpedit_replay_t *r, void *out, size_t cap, size_t *out_len)
{
    if (!t || !r || !out || !out_len)
        return TCPEDIT_ERROR;
    *out_len = 0;
    const int cached = r->preload && r->pass > 0;
    if (r->list.n && !r->list_set && replay_set_list(t, r) < 0)
        return TCPEDIT_ERROR;
    if (cached && tcpedit_batch_update_input(t, r->b, r->cache, r->len) < 0)
        return TCPEDIT_ERROR;
    const int rc = tcpedit_batch_run(t, r->b);
    tcpedit_batch_result_t res;
    if (tcpedit_batch_result(r->b, &res) < 0)
        return TCPEDIT_ERROR;
    if (cached && res.stale_records) {
        te_seterr(t, "tcpedit_replay: a record's edit reads its --preload-pcap cache buffer past its bytes "
                     "(SURVEY Q8): not reproduced");
        return TCPEDIT_ERROR;
    }
    const uint8_t *st = tcpedit_batch_status(r->b);
    uint8_t *o = malloc(res.out_len > 24 ? res.out_len : 24);
    if (!o || !st) {
        free(o);
        te_seterr(t, "tcpedit_replay: out of memory");
        return TCPEDIT_ERROR;
    }
    const size_t olen = tcpedit_batch_output(r->b, o, res.out_len);
    const uint8_t *src = cached ? r->cache : r->img;
    /* --unique-ip this pass (send_packets.c:477): the edited records' places in the batch
       output, their fast_edit_packet on the device */
    const int uedit = r->unique_ip && r->uniq && r->uniq > r->last_uniq;
    uint64_t *uoff = NULL, *usize = NULL, nu = 0;
    uint32_t *upatch = NULL;
    if (uedit) {
        uoff = malloc(8 * (r->nrec + 1));
        usize = malloc(8 * (r->nrec + 1));
        upatch = malloc(16 * (r->nrec + 1));
        if (!uoff || !usize || !upatch) {
            free(uoff);
            free(usize);
            free(upatch);
            free(o);
            te_seterr(t, "tcpedit_replay: out of memory");
            return TCPEDIT_ERROR;
        }
        for (uint64_t i = 0, q = 24; i < r->nrec && q + 16 <= olen; i++) {
            if ((st[i] & TE_ST_RC_MASK) == TE_ST_RC_ERROR)
                break;
            if (st[i] & TE_ST_ZEROCAP)
                continue;
            if (!(st[i] & TE_ST_NOSEND))
                uoff[nu++] = q;
            q += 16 + rp32(o + q + 8, 0);
        }
        if (nu && replay_unique(t, r, uoff, nu, usize, upatch) < 0) {
            free(uoff);
            free(usize);
            free(upatch);
            free(o);
            return TCPEDIT_ERROR;
        }
    }
    /* the records as sent: every record edited (one the edit emptied too: pcap_dump writes
       it, where tcprewrite drops it, tcprewrite.c:367), its fraction as the dump writes it */
    size_t ip = 24, op = 24, w = 0;
    uint64_t ku = 0;
    int err = 0;
    for (uint64_t i = 0; i < r->nrec; i++) {
        const uint32_t frac = rp32(src + ip + 4, r->swapped), cl0 = rp32(src + ip + 8, r->swapped);
        if ((st[i] & TE_ST_RC_MASK) == TE_ST_RC_ERROR) {
            err = 1;
            break;
        }
        if (st[i] & TE_ST_NOSEND) { /* the list left it out: written unedited to the batch output */
            if (!(st[i] & TE_ST_ZEROCAP))
                op += 16 + rp32(o + op + 8, 0);
            ip += 16 + cl0;
            continue;
        }
        uint32_t h[4];
        if (st[i] & TE_ST_ZEROCAP) {
            /* a record with caplen 0 after its edit (the batch output leaves it out): no
               record is read that way (safe_pcap_next exits, utils.c:147-156), so the edit
               emptied it -- the fuzz step's drop (fuzzing.c:37-60: caplen = len = 0) */
            h[0] = rp32(src + ip, r->swapped);
            h[2] = 0;
            h[3] = 0;
        } else {
            if (op + 16 > olen) { /* (the batch wrote fewer records than it edited) */
                err = 1;
                te_seterr(t, "tcpedit_replay: record %llu missing from the batch output", (unsigned long long)i + 1);
                break;
            }
            memcpy(h, o + op, 16);
        }
        h[1] = r->nsec ? frac : frac * 1000u;
        const uint32_t *pt = NULL; /* this record's unique-ip patch */
        if (uedit) {
            if ((st[i] & TE_ST_ZEROCAP) || !usize[ku]) { /* fast_edit_packet failed: not sent */
                r->failed++;
                if (!(st[i] & TE_ST_ZEROCAP)) {
                    ku++;
                    if (cached) /* (the edit of the cached bytes stands) */
                        memcpy(r->cache + ip + 16, o + op + 16, h[2] < cl0 ? h[2] : cl0);
                    op += 16 + h[2];
                }
                ip += 16 + cl0;
                continue;
            }
            pt = upatch + 4 * ku++;
        }
        if (w + 16 + h[2] > cap) {
            free(uoff);
            free(usize);
            free(upatch);
            free(o);
            te_seterr(t, "tcpedit_replay: record %llu: %u output bytes past the pass's buffer (%zu)",
                      (unsigned long long)i + 1, h[2], cap);
            return TCPEDIT_ERROR;
        }
        memcpy((uint8_t *)out + w, h, 16);
        if (!(st[i] & TE_ST_ZEROCAP)) {
            if (pt && pt[0]) { /* the new addresses into the edited bytes (at_s 0: unchanged) */
                put_be32(o + op + 16 + pt[0], pt[1]);
                put_be32(o + op + 16 + pt[2], pt[3]);
            }
            memcpy((uint8_t *)out + w + 16, o + op + 16, h[2]);
            if (cached) {
                /* the cache buffer after this edit (every pass but the first edits it in place;
                   the first edits libpcap's buffer and leaves the cache unedited): the edited
                   bytes, then past the edited length the bytes the edit did not touch */
                const uint32_t n = h[2] < cl0 ? h[2] : cl0;
                memcpy(r->cache + ip + 16, o + op + 16, n);
            }
            op += 16 + h[2];
        }
        w += 16 + h[2];
        ip += 16 + cl0;
    }
    free(uoff);
    free(usize);
    free(upatch);
    free(o);
    *out_len = w;
    r->pass++;
    /* increment_iteration (send_packets.c:362-372) */
    r->last_uniq = r->uniq;
    r->iteration++;
    if (r->unique_ip)
        r->uniq = (r->iteration * 1000) / (uint64_t)(r->unique_loops * 1000.0) + 1;
    return err || rc < 0 ? TCPEDIT_ERROR : TCPEDIT_OK;
}
