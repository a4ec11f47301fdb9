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
 * libpcap's nanosecond read leaves it).  Not served (refused): stale static-buffer reads
 *  on a cached pass (the reference reads its cache buffer's headroom there),
 * --fuzz-seed with -K over several passes, non-Ethernet captures (tcpreplay-edit decodes
 * with the interface's DLT, DLT_EN10MB for the dump).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/tcpedit.h"
#include "te_dev_cfg.h"
#include "te_internal.h"

struct tcpedit_replay_s {
    tcpedit_batch_t *b;
    uint8_t *img;     /* the capture (host copy) */
    uint8_t *cache;   /* -K: the cached records, same layout as img */
    size_t len;
    uint64_t nrec, pass;
    int preload, swapped, nsec;
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
    r->len = len;
    r->img = malloc(len);
    if (!r->img)
        goto fail;
    memcpy(r->img, pcap, len);
    for (size_t p = 24; p + 16 <= len; r->nrec++) { /* libpcap's walk */
        const uint32_t cl = rp32(r->img + p + 8, r->swapped);
        if (cl > 262144u || p + 16 + cl > len)
            break;
        p += 16 + cl;
    }
    if (preload) {
        r->cache = malloc(len);
        if (!r->cache)
            goto fail;
        memcpy(r->cache, pcap, len);
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
    tcpedit_batch_close(r->b);
    free(r->img);
    free(r->cache);
    free(r);
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
    /* the records as sent: every record edited (a zero-length one too: pcap_dump writes it,
       where tcprewrite drops it, tcprewrite.c:367), its fraction as the dump writes it */
    const uint8_t *src = cached ? r->cache : r->img;
    size_t ip = 24, op = 24, w = 0;
    int err = 0;
    for (uint64_t i = 0; i < r->nrec; i++) {
        const uint32_t frac = rp32(src + ip + 4, r->swapped), cl0 = rp32(src + ip + 8, r->swapped);
        if ((st[i] & TE_ST_RC_MASK) == TE_ST_RC_ERROR) {
            err = 1;
            break;
        }
        uint32_t h[4];
        if (st[i] & TE_ST_ZEROCAP) {
            /* a record read with caplen 0 (no edit step can empty one): tcpedit_packet's
               only change to it is --efcs's trim of len (tcpedit.c:78-84), then the L2 parse
               fails (a soft error) */
            const uint32_t ln = rp32(src + ip + 12, r->swapped);
            h[0] = rp32(src + ip, r->swapped);
            h[2] = 0;
            h[3] = ((const tcpedit_ref_t *)t)->efcs && ln > 4 ? ln - 4 : ln;
        } else {
            if (op + 16 > olen)
                break;
            memcpy(h, o + op, 16);
        }
        h[1] = r->nsec ? frac : frac * 1000u;
        if (w + 16 + h[2] > cap) {
            free(o);
            te_seterr(t, "tcpedit_replay: record %llu: %u output bytes past the pass's buffer (%zu)",
                      (unsigned long long)i + 1, h[2], cap);
            return TCPEDIT_ERROR;
        }
        memcpy((uint8_t *)out + w, h, 16);
        if (!(st[i] & TE_ST_ZEROCAP)) {
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
    free(o);
    *out_len = w;
    r->pass++;
    return err || rc < 0 ? TCPEDIT_ERROR : TCPEDIT_OK;
}
