/*
 * te_pcapng.c -- pcapng input as libpcap's reader hands it to tcprewrite (SURVEY Q0,
 * 8(f) rank 1).  tcprewrite reads with pcap_open_offline (tcprewrite.c:244-254) and
 * pcap_next (:289), which for a pcapng file are libpcap's pcap-ng reader: records come
 * out as classic pcap headers at microsecond precision, and tcprewrite writes a classic
 * pcap file.  So a pcapng image becomes the classic image the edit path reads:
 *
 *   SHB (0x0A0D0D0A)  byte order from its magic 0x1A2B3C4D; a later SHB starts a new
 *                     section (its interfaces replace the earlier ones)
 *   IDB (1)           linktype, snaplen, if_tsresol (option 9), if_tsoffset (option 14)
 *   EPB (6)           interface, 64-bit timestamp, captured / original length, data
 *   SPB (3)           original length; captured = min(original, the snapshot length)
 *   OPB (2, obsolete) interface (16 bits), drops, timestamp, lengths, data
 *   others            skipped (name resolution, statistics, secrets, custom blocks)
 *
 * Timestamps are converted to seconds and microseconds as libpcap does: units per second
 * from if_tsresol (10^n, or 2^n with the high bit), if_tsoffset added to the seconds, the
 * fraction scaled to microseconds (truncating).  Every interface must have the first
 * one's link type (libpcap refuses a file that mixes them).  The capture's snapshot
 * length is the first interface's snaplen (0, or more than 262144, meaning 262144, as
 * pcap_adjust_snapshot has it), and a record's captured length is cut to it.
 * Parity is unpinned: the reference holds no pcapng fixture; tests/test_pcapng.py checks
 * the conversion against the classic capture a pcapng file was written from.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "te_internal.h"

#define NG_MAX_IF 256

typedef struct {
    uint32_t linktype, snaplen;
    uint64_t units;  /* timestamp units per second */
    int64_t offset;  /* if_tsoffset, seconds */
} ng_if_t;

static uint32_t ng32(const uint8_t *p, int sw)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

static uint16_t ng16(const uint8_t *p, int sw)
{
    uint16_t v;
    memcpy(&v, p, 2);
    return sw ? __builtin_bswap16(v) : v;
}

int te_is_pcapng(const uint8_t *img, size_t len)
{
    uint32_t m;
    if (len < 4)
        return 0;
    memcpy(&m, img, 4);
    return m == 0x0A0D0D0Au;
}

static int ng_err(char *err, size_t errlen, const char *msg)
{
    if (err && errlen)
        snprintf(err, errlen, "%s", msg);
    return -1;
}

/* the interface's option list: if_tsresol, if_tsoffset */
static void ng_if_options(const uint8_t *o, const uint8_t *end, int sw, ng_if_t *f)
{
    while (o + 4 <= end) {
        const uint16_t code = ng16(o, sw), olen = ng16(o + 2, sw);
        const uint8_t *v = o + 4;
        if (code == 0 || v + olen > end)
            break;
        if (code == 9 && olen >= 1) { /* if_tsresol */
            const uint8_t r = v[0];
            uint64_t u = 1;
            if (r & 0x80) {
                const int p = r & 0x7f;
                u = p < 64 ? (1ull << p) : 0;
            } else {
                for (int i = 0; i < (r & 0x7f) && u; i++)
                    u = u > UINT64_MAX / 10 ? 0 : u * 10;
            }
            if (u)
                f->units = u;
        } else if (code == 14 && olen >= 8) { /* if_tsoffset */
            uint64_t x;
            memcpy(&x, v, 8);
            f->offset = (int64_t)(sw ? __builtin_bswap64(x) : x);
        }
        o = v + ((olen + 3u) & ~3u);
    }
}

/* one record into the classic image */
static int ng_put(uint8_t **out, size_t *n, size_t *cap, const ng_if_t *f, uint64_t ts, uint32_t caplen,
                  uint32_t origlen, const uint8_t *data)
{
    if (*n + 16 + caplen > *cap) {
        size_t c = *cap * 2;
        while (c < *n + 16 + caplen)
            c *= 2;
        uint8_t *g = realloc(*out, c);
        if (!g)
            return -1;
        *out = g;
        *cap = c;
    }
    const uint64_t u = f->units;
    const uint64_t frac = ts % u;
    const uint64_t usec = (uint64_t)((unsigned __int128)frac * 1000000 / u); /* truncating, as the scalings */
    const uint64_t sec = (uint64_t)((int64_t)(ts / u) + f->offset);
    const uint32_t h[4] = {(uint32_t)sec, (uint32_t)usec, caplen, origlen};
    memcpy(*out + *n, h, 16);
    memcpy(*out + *n + 16, data, caplen);
    *n += 16 + caplen;
    return 0;
}

int te_pcapng_to_pcap(const uint8_t *in, size_t len, uint8_t **out_img, size_t *out_len, char *err, size_t errlen)
{
    *out_img = NULL;
    *out_len = 0;
    if (!te_is_pcapng(in, len) || len < 28)
        return ng_err(err, errlen, "not a pcapng file");
    size_t cap = len + 64, n = 24;
    uint8_t *out = malloc(cap);
    if (!out)
        return ng_err(err, errlen, "out of host memory");
    ng_if_t *ifs = calloc(NG_MAX_IF, sizeof *ifs);
    if (!ifs) {
        free(out);
        return ng_err(err, errlen, "out of host memory");
    }
    int nif = 0, sw = 0;
    uint32_t linktype = 0, snaplen = 0, snapshot = 262144u;
    int have_link = 0;
    size_t p = 0;
    while (p + 12 <= len) {
        uint32_t type;
        memcpy(&type, in + p, 4);
        if (type == 0x0A0D0D0Au) { /* SHB: byte order, a new section */
            uint32_t bom;
            memcpy(&bom, in + p + 8, 4);
            if (bom == 0x1A2B3C4Du)
                sw = 0;
            else if (bom == 0x4D3C2B1Au)
                sw = 1;
            else
                goto bad;
            nif = 0;
        } else {
            type = ng32(in + p, sw);
        }
        const uint32_t blen = ng32(in + p + 4, sw);
        if (blen < 12 || blen % 4 || p + blen > len)
            break; /* a truncated last block: libpcap's reader stops */
        const uint8_t *b = in + p + 8, *bend = in + p + blen - 4;
        if (type == 1) { /* IDB */
            if (b + 8 > bend || nif >= NG_MAX_IF)
                goto bad;
            ng_if_t f = {ng16(b, sw), ng32(b + 4, sw), 1000000, 0};
            ng_if_options(b + 8, bend, sw, &f);
            if (!have_link) {
                linktype = f.linktype;
                snaplen = f.snaplen;
                /* pcap_adjust_snapshot: 0 or more than the maximum means the maximum */
                snapshot = (snaplen == 0 || snaplen > 262144u) ? 262144u : snaplen;
                have_link = 1;
            } else if (f.linktype != linktype) {
                free(out);
                free(ifs);
                return ng_err(err, errlen, "pcapng: an interface has a link type different from the first one's");
            }
            ifs[nif++] = f;
        } else if (type == 6 || type == 2) { /* EPB / OPB */
            if (b + 20 > bend)
                goto bad;
            const uint32_t ifn = type == 6 ? ng32(b, sw) : ng16(b, sw);
            const uint64_t ts = (uint64_t)ng32(b + 4, sw) << 32 | ng32(b + 8, sw);
            const uint32_t cl = ng32(b + 12, sw), ol = ng32(b + 16, sw);
            /* unsigned compares: an interface id or length read from the file never indexes
               or reaches past what the block holds */
            if (ifn >= (uint32_t)nif || (size_t)cl > (size_t)(bend - (b + 20)))
                goto bad;
            /* libpcap's reader cuts a record to the capture's snapshot length */
            if (ng_put(&out, &n, &cap, &ifs[ifn], ts, cl > snapshot ? snapshot : cl, ol, b + 20) < 0)
                goto oom;
        } else if (type == 3) { /* SPB: interface 0, no timestamp */
            if (b + 4 > bend || nif < 1)
                goto bad;
            const uint32_t ol = ng32(b, sw);
            uint32_t cl = ol > snapshot ? snapshot : ol;
            if ((size_t)cl > (size_t)(bend - (b + 4)))
                cl = (uint32_t)(bend - (b + 4));
            if (ng_put(&out, &n, &cap, &ifs[0], 0, cl, ol, b + 4) < 0)
                goto oom;
        }
        p += blen;
    }
    if (!have_link) {
        free(out);
        free(ifs);
        return ng_err(err, errlen, "pcapng: no interface description block");
    }
    { /* the classic header: LE, microseconds, the interfaces' link type and first snaplen */
        const uint32_t h[6] = {0xa1b2c3d4u, 2u | 4u << 16, 0, 0, snaplen ? snaplen : 262144u, linktype};
        memcpy(out, h, 24);
    }
    free(ifs);
    *out_img = out;
    *out_len = n;
    return 0;
bad:
    free(out);
    free(ifs);
    return ng_err(err, errlen, "pcapng: malformed block");
oom:
    free(out);
    free(ifs);
    return ng_err(err, errlen, "out of host memory");
}

int tcpedit_pcapng_to_pcap(const void *in, size_t len, void **out, size_t *out_len)
{
    if (!in || !out || !out_len)
        return -1;
    uint8_t *o = NULL;
    const int rc = te_pcapng_to_pcap(in, len, &o, out_len, NULL, 0);
    *out = o;
    return rc;
}
