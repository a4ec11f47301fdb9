/*
 * tcpreplay_oracle.c -- CPU restatement of tcpreplay's file-output replay with
 * --unique-ip (TEST INFRASTRUCTURE ONLY: tests/, bench.py's cpu_baseline and
 * __graft_entry__.smoke() use it as the checker; the product never links it).
 * Included by tcpprep_oracle.c (one liboracle.so, shared L2 locator).
 *
 *   tcpreplay -w <file> [-K] [--loop=N] [--unique-ip [--unique-ip-loops=L]] <pcap>
 *
 * follows:
 *   send_packets        src/send_packets.c:379-646  (one pass over the capture; a record
 *                       whose unique-ip edit fails is counted and not sent, :477-483)
 *   increment_iteration src/send_packets.c:362-372  (after every pass)
 *   fast_edit_packet    src/send_packets.c:124-257  (src/dst address shift, no checksum
 *                       change; COUNTER arithmetic is 64-bit)
 *   the -w dump         src/common/sendpacket.c:485-486,945-968: pcap_open_dead(DLT_EN10MB,
 *                       MAX_SNAPLEN) + pcap_dump, each record's header as read
 *   the read            libpcap opened with nanosecond precision: the timestamp fraction
 *                       of a microsecond capture is scaled by 1000, and pcap_dump writes that
 *                       value into the microsecond file (test2.replay_unique_ip holds it)
 * Parity pinned: test/test2.replay_unique_ip (tests/golden).
 */

/* fast_edit_packet (send_packets.c:124-257) over one packet; -1: not edited (not sent) */
static int tro_fast_edit(uint8_t *pkt, uint32_t caplen, uint64_t iteration, int cached)
{
    uint16_t proto = 0;
    uint32_t l2len = 0, l2off = 0, voff = 0;
    if (get_l2len_protocol(pkt, caplen, &proto, &l2len, &l2off, &voff) < 0)
        return -1;
    uint8_t *s_at, *d_at;
    if (proto == 0x0800) {
        if (caplen < l2len + 20)
            return -1;
        s_at = pkt + l2len + 12;
        d_at = pkt + l2len + 16;
    } else if (proto == 0x86DD) {
        if (caplen < l2len + 40)
            return -1;
        s_at = pkt + l2len + 8 + 12; /* ip_src.__u6_addr32[3] */
        d_at = pkt + l2len + 24 + 12;
    } else {
        return -1;
    }
    const uint32_t so = (uint32_t)s_at[0] << 24 | (uint32_t)s_at[1] << 16 | (uint32_t)s_at[2] << 8 | s_at[3];
    const uint32_t dor = (uint32_t)d_at[0] << 24 | (uint32_t)d_at[1] << 16 | (uint32_t)d_at[2] << 8 | d_at[3];
    uint32_t src = so, dst = dor;
    if ((!cached && dst > src) || (cached && ((uint64_t)dst - iteration) > ((uint64_t)src - 1 - iteration))) {
        if (cached) {
            --src;
            ++dst;
        } else {
            src -= (uint32_t)iteration;
            dst += (uint32_t)iteration;
        }
        if (src > so && dst > dor)
            --src;
        else if (dst < dor && src < so)
            ++dst;
    } else {
        if (cached) {
            ++src;
            --dst;
        } else {
            src += (uint32_t)iteration;
            dst -= (uint32_t)iteration;
        }
        if (dst > dor && src > so)
            --dst;
        else if (src < so && dst < dor)
            ++src;
    }
    for (int k = 0; k < 4; k++) {
        s_at[k] = (uint8_t)(src >> (24 - 8 * k));
        d_at[k] = (uint8_t)(dst >> (24 - 8 * k));
    }
    return 0;
}

/* the --include / --exclude packet list (tcpreplay_opts.def:305-360):
 *   parse_list  src/common/list.c:61-130 -- ',' tokens (strtok_r: empty ones vanish), each
 *               matching "^[0-9]+(-([0-9]+|\s*))?$"; add_to_list (:36-50): min by
 *               strtoull(.., 0), max = min without '-', 0 for "N-" (open), else strtoull
 *   check_list  src/common/list.c:139-156 -- min and max set: min <= v <= max; min 0:
 *               v <= max; max 0: v >= min
 * A list that does not parse is the reference's errx ("Unable to parse include/exclude
 * rule"): -1 here. */
typedef struct {
    uint64_t min[4096], max[4096];
    int n;
} tro_list_t;

static int tro_list_parse(tro_list_t *l, const char *arg)
{
    char buf[16384];
    if (!arg || strlen(arg) >= sizeof buf)
        return -1;
    strcpy(buf, arg);
    l->n = 0;
    char *tok = NULL;
    for (char *e = strtok_r(buf, ",", &tok); e; e = strtok_r(NULL, ",", &tok)) {
        char *p = e, *second = NULL;
        if (!isdigit((unsigned char)*p))
            return -1;
        while (isdigit((unsigned char)*p))
            p++;
        if (*p == '-') {
            *p++ = 0;
            second = p;
            if (isdigit((unsigned char)*p))
                while (isdigit((unsigned char)*p))
                    p++;
            else
                while (*p == ' ' || (*p >= '\t' && *p <= '\r'))
                    p++;
        }
        if (*p || l->n >= 4096)
            return -1;
        l->min[l->n] = strtoull(e, NULL, 0);
        l->max[l->n] = second ? (second[0] ? strtoull(second, NULL, 0) : 0) : l->min[l->n];
        l->n++;
    }
    return l->n ? 0 : -1;
}

static int tro_list_check(const tro_list_t *l, uint64_t v)
{
    for (int i = 0; i < l->n; i++) {
        const uint64_t mn = l->min[i], mx = l->max[i];
        if (mn != 0 && mx != 0) {
            if (v >= mn && v <= mx)
                return 1;
        } else if (mn == 0) {
            if (v <= mx)
                return 1;
        } else if (mx == 0) {
            if (v >= mn)
                return 1;
        }
    }
    return 0;
}

/* send_packets.c:440-447: a record the list leaves out is skipped before anything else
   (no edit, not sent, not counted) */
static int tro_listed_out(const tro_list_t *l, int exclude, uint64_t packetnum)
{
    if (!l)
        return 0;
    const int rule_set = tro_list_check(l, packetnum);
    return (rule_set && exclude) || (!rule_set && !exclude);
}

/* 1 when the last run ended at safe_pcap_next's exit(-1) (its length: the records before) */
static int g_replay_exit;
int tcpreplay_oracle_exited(void) { return g_replay_exit; }

/* returns the output length, or -1 bad options, -2 not a pcap, -3 out too small */
long tcpreplay_oracle_run_list(const uint8_t *pcap, size_t len, int loops, int unique_ip, double unique_loops,
                               int preload, const char *list, int exclude, uint8_t *out, size_t cap,
                               uint64_t *failed);
long tcpreplay_oracle_run(const uint8_t *pcap, size_t len, int loops, int unique_ip, double unique_loops,
                          int preload, uint8_t *out, size_t cap, uint64_t *failed)
{
    return tcpreplay_oracle_run_list(pcap, len, loops, unique_ip, unique_loops, preload, NULL, 0, out, cap, failed);
}

long tcpreplay_oracle_run_list(const uint8_t *pcap, size_t len, int loops, int unique_ip, double unique_loops,
                               int preload, const char *list, int exclude, uint8_t *out, size_t cap,
                               uint64_t *failed)
{
    static tro_list_t lst;
    if (loops < 1 || (unique_ip && unique_loops < 1.0))
        return -1;
    if (list && tro_list_parse(&lst, list) < 0)
        return -1;
    if (len < 24)
        return -2;
    uint32_t magic;
    memcpy(&magic, pcap, 4);
    int sw, nsec;
    if (magic == 0xa1b2c3d4u || magic == 0xd4c3b2a1u)
        nsec = 0;
    else if (magic == 0xa1b23c4du || magic == 0x4d3cb2a1u)
        nsec = 1;
    else
        return -2;
    sw = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    if (cap < 24)
        return -3;
    /* pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN) + pcap_dump_open */
    static const uint8_t hdr[24] = {0xd4, 0xc3, 0xb2, 0xa1, 2, 0, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 4, 0, 1, 0, 0, 0};
    memcpy(out, hdr, 24);
    size_t o = 24;
    uint8_t *cache = NULL; /* -K: the records, edited in place from pass to pass */
    if (preload) {
        cache = malloc(len);
        if (!cache)
            return -3;
        memcpy(cache, pcap, len);
    }
    static uint8_t pkt[MAXPACKET + 64];
    uint64_t iteration = 0, uniq = 0, last_uniq = 0;
    *failed = 0;
    g_replay_exit = 0;
    for (int pass = 0; pass < loops; pass++) {
        uint64_t packetnum = 0;
        size_t off = 24, dat = 0;
        uint32_t caplen = 0;
        int nx;
        /* get_next_packet (send_packets.c:955,985): safe_pcap_next's reader rules (tpo_next);
           its exit(-1) comes in the first pass, with the records sent so far in the file */
        while ((nx = tpo_next(pcap, len, sw, &off, &dat, &caplen)) != 0) {
            if (nx < 0) {
                g_replay_exit = 1;
                free(cache);
                return (long)o;
            }
            const uint32_t ts = tpo_rd32(pcap + dat - 16, sw), frac = tpo_rd32(pcap + dat - 12, sw);
            const uint32_t plen = tpo_rd32(pcap + dat - 4, sw);
            uint8_t *data = preload ? cache + dat : pkt;
            if (!preload)
                memcpy(pkt, pcap + dat, caplen);
            if (tro_listed_out(list ? &lst : NULL, exclude, ++packetnum))
                continue;
            if (unique_ip && uniq && uniq > last_uniq && tro_fast_edit(data, caplen, uniq - 1, preload) == -1) {
                ++*failed;
                continue;
            }
            if (o + 16 + caplen > cap) {
                free(cache);
                return -3;
            }
            const uint32_t f = nsec ? frac : frac * 1000u;
            const uint32_t h[4] = {ts, f, caplen, plen};
            memcpy(out + o, h, 16);
            memcpy(out + o + 16, data, caplen);
            o += 16 + caplen;
        }
        /* increment_iteration */
        last_uniq = uniq;
        ++iteration;
        if (unique_ip)
            uniq = (iteration * 1000) / (uint64_t)(unique_loops * 1000.0) + 1;
    }
    free(cache);
    return (long)o;
}

static uint64_t g_replay_failed;

/* CPU restatement of tcpreplay-edit's send loop with file output (test infrastructure):
 *   main                tcpreplay.c:79-100: tcpedit_init(sendpacket_get_dlt(intf1)) -- the
 *                       -w dump interface is DLT_EN10MB (sendpacket.c:945-968) --,
 *                       tcpedit_post_args, tcpedit_validate
 *   send_packets        send_packets.c:379-640: per record, tcpedit_packet(ctx, &hdr, &data,
 *                       intf1's direction TCPR_DIR_C2S) (:469-474; -1 ends the run, errx);
 *                       the packet is sent as edited, soft errors included
 *   get_next_packet     send_packets.c:918-990: without -K every pass reads the file through
 *                       libpcap (one reused read buffer, zeroed when first mapped); with -K
 *                       the first pass still edits libpcap's buffer while caching an unedited
 *                       copy of every record (caplen + PACKET_HEADROOM 512 zeroed bytes,
 *                       defines.h.in:184) and its header, and every later pass edits the
 *                       cached bytes IN PLACE with a copy of the cached header: edits
 *                       compound from pass to pass
 *   the -w dump         sendpacket.c:485-486: pcap_dump of the edited header and bytes into
 *                       pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN) (the fraction as libpcap's
 *                       nanosecond read leaves it: x1000 for a microsecond capture)
 * Parity unpinned: the reference holds no tcpreplay-edit output fixture.  Refused here as on
 * the device: --fuzz-seed with -K (fuzz writes land in the cache headroom). */
int tcpreplay_edit_oracle_run(const uint8_t *in, size_t in_len, int loops, int preload, int argc, const char **argv,
                              uint8_t *out, size_t out_cap, size_t *out_len, char *errbuf, int errlen)
{
    oopts_t *o = calloc(1, sizeof(oopts_t));
    ocfg_t c;
    int rc = 0;
    size_t op = 24;
    uint8_t *buf = NULL, **cache = NULL;
    uint32_t *chdr = NULL;
    uint64_t nrec = 0;
    memset(&c, 0, sizeof(c));
    g_err[0] = 0;
    /* tcpreplay's own options on this path; the rest are tcpedit's */
    static tro_list_t lst;
    const char *list = NULL;
    int exclude = 0, unique_ip = 0;
    double unique_loops = 1.0;
    const char **targv = calloc((size_t)argc + 1, sizeof(*targv));
    int targc = 0;
    for (int i = 0; i < argc; i++) {
        const char *a = argv[i];
        if (!strncmp(a, "--include=", 10) || !strncmp(a, "--exclude=", 10)) {
            if (list) { /* flags-cant: include and exclude exclude each other (max 1) */
                seterr("--include and --exclude: only one list");
                rc = -2;
                goto out;
            }
            exclude = a[2] == 'e';
            list = a + 10;
        } else if (!strcmp(a, "--unique-ip")) {
            unique_ip = 1;
        } else if (!strncmp(a, "--unique-ip-loops=", 18)) {
            unique_loops = atof(a + 18);
        } else {
            targv[targc++] = a;
        }
    }
    if (list && tro_list_parse(&lst, list) < 0) {
        seterr("Unable to parse include/exclude rule: %s", list);
        rc = -2;
        goto out;
    }
    if (unique_ip && unique_loops < 1.0) {
        seterr("--unique-ip-loops requires loop count >= 1.0");
        rc = -2;
        goto out;
    }
    uint64_t iteration = 0, uniq = 0, last_uniq = 0, nfailed = 0;
    c.decoder = DEC_EN10MB;
    c.in_dlt = 1;
    if (loops < 1 || in_len < 24 || out_cap < 24) {
        seterr("bad arguments");
        rc = -2;
        goto out;
    }
    if (parse_argv(o, targc, targv) < 0 || oracle_post_args(&c, o) < 0) {
        rc = -2;
        goto out;
    }
    if (c.fuzz_seed && preload) {
        seterr("--fuzz-seed with --preload-pcap is not served");
        rc = -2;
        goto out;
    }
    uint32_t magic;
    memcpy(&magic, in, 4);
    const int swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    const int nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    if (!swap && !nsec && magic != 0xa1b2c3d4u) {
        seterr("bad pcap magic");
        rc = -2;
        goto out;
    }
    {
        const uint32_t hdr[6] = {0xa1b2c3d4u, 0x00040002u, 0, 0, 262144u, 1u};
        memcpy(out, hdr, 24);
    }
    buf = calloc(1, MAXPACKET + 65536); /* libpcap's read buffer (a fresh mapping: zero) */
    /* the records (libpcap's walk, then safe_pcap_next, send_packets.c:955,985 ->
       src/common/utils.c:131-169): a record with len > MAX_SNAPLEN or a zero len or caplen
       exit(-1)s when the first pass reaches it */
    int reader_exit = 0;
    {
        size_t p = 24, d = 0;
        uint32_t cl = 0;
        int nx;
        while ((nx = tpo_next(in, in_len, swap, &p, &d, &cl)) > 0)
            nrec++;
        reader_exit = nx < 0;
    }
    if (preload) {
        cache = calloc(nrec ? nrec : 1, sizeof(*cache));
        chdr = calloc(nrec ? 4 * nrec : 1, sizeof(*chdr));
    }
    ostate_t st;
    memset(&st, 0, sizeof(st));
    g_fuzz_state = c.fuzz_seed;
    g_fuzz_draws = 0;
    g_fuzz_factor = c.fuzz_factor ? c.fuzz_factor : 8;
    for (int pass = 0; pass < loops && rc == 0; pass++) {
        size_t p = 24;
        for (uint64_t i = 0; i < nrec; i++) {
            const int listed_out = tro_listed_out(list ? &lst : NULL, exclude, i + 1); /* :440-447 */
            uint32_t rh[4];
            memcpy(rh, in + p, 16);
            if (swap)
                for (int q = 0; q < 4; q++)
                    rh[q] = bswap32_(rh[q]);
            const uint32_t file_cap = rh[2];
            if (rh[3] < rh[2]) /* utils.c:159-162: caplen = len */
                rh[2] = rh[3];
            uint8_t *data;
            ohdr_t h = {rh[2], rh[3]};
            if (!preload || pass == 0) {
                memcpy(buf, in + p + 16, rh[2]);
                data = buf;
                if (preload) { /* the unedited copy and header the later passes use (:973-977) */
                    cache[i] = calloc(1, (size_t)rh[2] + 512 + 4096);
                    memcpy(cache[i], in + p + 16, rh[2]);
                    memcpy(chdr + 4 * i, rh, 16);
                }
            } else {
                data = cache[i];
                h.caplen = chdr[4 * i + 2];
                h.len = chdr[4 * i + 3];
            }
            p += 16 + file_cap;
            if (listed_out)
                continue; /* read (and cached under -K), not edited, not sent */
            int warned = 0;
            const int prc = oracle_tcpedit_packet(&c, &st, &h, data, DIR_C2S, &warned);
            if (prc == TCPEDIT_ERROR) {
                seterr("Error editing packet #%llu", (unsigned long long)(i + 1));
                rc = -1;
                break;
            }
            if (preload && pass > 0 && h.caplen > chdr[4 * i + 2] + 512) {
                seterr("record %llu grows past the preload cache's headroom", (unsigned long long)(i + 1));
                rc = -2;
                break;
            }
            /* --unique-ip (:477-483): fast_edit_packet of the edited packet, with the header
               as read; a record it fails is counted and not sent */
            if (unique_ip && uniq && uniq > last_uniq &&
                tro_fast_edit(data, h.caplen, uniq - 1, preload && pass > 0) == -1) {  /* the edited header */
                ++nfailed;
                continue;
            }
            if (op + 16 + h.caplen > out_cap) {
                seterr("output buffer too small");
                rc = -2;
                break;
            }
            const uint32_t f = nsec ? rh[1] : rh[1] * 1000u;
            const uint32_t orh[4] = {rh[0], f, h.caplen, h.len};
            memcpy(out + op, orh, 16);
            memcpy(out + op + 16, data, h.caplen);
            op += 16 + h.caplen;
        }
        if (rc == 0 && pass == 0 && reader_exit) {
            seterr("safe_pcap_next ERROR: Invalid packet length: packet %llu", (unsigned long long)(nrec + 1));
            rc = -1;
        }
        /* increment_iteration (send_packets.c:362-372) */
        last_uniq = uniq;
        ++iteration;
        if (unique_ip)
            uniq = (iteration * 1000) / (uint64_t)(unique_loops * 1000.0) + 1;
    }
    g_replay_failed = nfailed;
    *out_len = op; /* (-1: the records sent before the error) */
out:
    if (errbuf && errlen > 0)
        snprintf(errbuf, (size_t)errlen, "%s", g_err);
    if (cache)
        for (uint64_t i = 0; i < nrec; i++)
            free(cache[i]);
    free(cache);
    free(chdr);
    free(buf);
    free_cfg(&c);
    free(o);
    free(targv);
    return rc;
}

/* records whose --unique-ip edit failed in the last tcpreplay_edit_oracle_run */
uint64_t tcpreplay_edit_oracle_failed(void) { return g_replay_failed; }
