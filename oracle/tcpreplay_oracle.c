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

/* returns the output length, or -1 bad options, -2 not a pcap, -3 out too small */
long tcpreplay_oracle_run(const uint8_t *pcap, size_t len, int loops, int unique_ip, double unique_loops,
                          int preload, uint8_t *out, size_t cap, uint64_t *failed)
{
    if (loops < 1 || (unique_ip && unique_loops < 1.0))
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
    for (int pass = 0; pass < loops; pass++) {
        for (size_t off = 24; off + 16 <= len;) {
            const uint32_t ts = tpo_rd32(pcap + off, sw), frac = tpo_rd32(pcap + off + 4, sw);
            const uint32_t caplen = tpo_rd32(pcap + off + 8, sw), plen = tpo_rd32(pcap + off + 12, sw);
            if (caplen > 262144u || off + 16 + caplen > len)
                break; /* libpcap stops */
            uint8_t *data = preload ? cache + off + 16 : pkt;
            if (!preload)
                memcpy(pkt, pcap + off + 16, caplen);
            off += 16 + caplen;
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
