"""Synthetic pcap workloads for the BASELINE.json configs.

All frames are Ethernet II, dst MAC 00:11:22:33:44:55, src MAC 00:66:77:88:99:aa,
valid IPv4/IPv6 and TCP/UDP checksums, IP length == caplen - 14 (so --fixcsum
really recomputes), sequential timestamps, little-endian microsecond pcap with
snaplen 65535.  Generation is vectorised with numpy so 10M-record IMIX files
build in seconds.
"""
import numpy as np

DST_MAC = bytes.fromhex("001122334455")
SRC_MAC = bytes.fromhex("00667788 99aa".replace(" ", ""))
IMIX_PATTERN = [64] * 7 + [570] * 4 + [1514]  # 7:4:1, deterministic order

PCAP_HDR = np.frombuffer(bytes.fromhex("d4c3b2a1020004000000000000000000ffff000001000000"), np.uint8)


def _fold(s):
    s = s.astype(np.uint64)
    while True:
        hi = s >> np.uint64(16)
        if not hi.any():
            break
        s = (s & np.uint64(0xFFFF)) + hi
    return s.astype(np.uint32)


def _sum16(a):
    """one's-complement sum (unfolded) of big-endian 16-bit words of each row (even widths)."""
    w = a.view(">u2").astype(np.uint64)
    return w.sum(axis=1)


def _frames(rng, n, size, ipv6=False, proto=17, first_index=0):
    """n frames of `size` bytes (caplen = len = size) as an (n, size) uint8 array."""
    f = np.empty((n, size), np.uint8)
    f[:, 0:6] = np.frombuffer(DST_MAC, np.uint8)
    f[:, 6:12] = np.frombuffer(SRC_MAC, np.uint8)
    idx = np.arange(first_index, first_index + n, dtype=np.uint64)
    sport = rng.integers(1024, 65535, n, dtype=np.uint32)
    dchoice = rng.integers(0, 5, n)
    dport = np.choose(dchoice, [np.full(n, 53), np.full(n, 80), np.full(n, 443), np.full(n, 8080),
                                rng.integers(1, 65535, n)]).astype(np.uint32)
    if not ipv6:
        f[:, 12:14] = (0x08, 0x00)
        ip = f[:, 14:34]
        ip[:, 0] = 0x45
        ip[:, 1] = 0
        tot = size - 14
        ip[:, 2], ip[:, 3] = (tot >> 8) & 0xFF, tot & 0xFF
        ident = (idx & np.uint64(0xFFFF)).astype(np.uint32)
        ip[:, 4], ip[:, 5] = ident >> 8, ident & 0xFF
        ip[:, 6] = 0x40  # DF
        ip[:, 7] = 0
        ip[:, 8] = 64
        ip[:, 9] = proto
        ip[:, 10:12] = 0
        src = (np.uint32(10) << 24) | rng.integers(0, 1 << 24, n, dtype=np.uint32)
        dst = (np.uint32(172 << 24) | np.uint32(16 << 16)) | rng.integers(0, 1 << 16, n, dtype=np.uint32)
        for k in range(4):
            ip[:, 12 + k] = (src >> np.uint32(24 - 8 * k)) & 0xFF
            ip[:, 16 + k] = (dst >> np.uint32(24 - 8 * k)) & 0xFF
        l4off = 34
        l4len = size - 34
    else:
        f[:, 12:14] = (0x86, 0xDD)
        ip = f[:, 14:54]
        ip[:, 0] = 0x60
        ip[:, 1:4] = 0
        pl = size - 54
        ip[:, 4], ip[:, 5] = (pl >> 8) & 0xFF, pl & 0xFF
        ip[:, 6] = proto
        ip[:, 7] = 64
        ip[:, 8:24] = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        ip[:, 8:10] = (0x20, 0x01)
        ip[:, 24:40] = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        ip[:, 24:26] = (0x20, 0x01)
        l4off = 54
        l4len = size - 54
    l4 = f[:, l4off:]
    l4[:] = rng.integers(0, 256, l4.shape, dtype=np.uint8)
    l4[:, 0], l4[:, 1] = sport >> 8, sport & 0xFF
    l4[:, 2], l4[:, 3] = dport >> 8, dport & 0xFF
    if proto == 17:
        l4[:, 4], l4[:, 5] = (l4len >> 8) & 0xFF, l4len & 0xFF
        ck = 6
    else:  # TCP: data offset 5, ACK|PSH
        l4[:, 12] = 0x50
        l4[:, 13] = 0x18
        l4[:, 14:16] = (0xFF, 0xFF)
        l4[:, 18:20] = 0
        ck = 16
    l4[:, ck:ck + 2] = 0
    # L4 checksum: pseudo header + segment (pad odd length with a zero byte)
    seg = l4 if l4len % 2 == 0 else np.concatenate([l4, np.zeros((n, 1), np.uint8)], axis=1)
    s = _sum16(seg)
    if not ipv6:
        s += _sum16(np.ascontiguousarray(ip[:, 12:20]))
    else:
        s += _sum16(np.ascontiguousarray(ip[:, 8:40]))
    s += np.uint64(proto + l4len)
    c = (~_fold(s)) & 0xFFFF
    if proto == 17:
        c = np.where(c == 0, 0xFFFF, c)
    l4[:, ck] = (c >> 8).astype(np.uint8)
    l4[:, ck + 1] = (c & 0xFF).astype(np.uint8)
    if not ipv6:
        hs = (~_fold(_sum16(np.ascontiguousarray(ip)))) & 0xFFFF
        ip[:, 10] = (hs >> 8).astype(np.uint8)
        ip[:, 11] = (hs & 0xFF).astype(np.uint8)
    return f


def _records(frames, ts0):
    """(n, size) frames -> (n, 16 + size) pcap records with sequential timestamps."""
    n, size = frames.shape
    r = np.empty((n, 16 + size), np.uint8)
    t = ts0 + np.arange(n, dtype=np.uint64)
    hdr = np.empty((n, 4), "<u4")
    hdr[:, 0] = 1600000000 + (t // np.uint64(1000000)).astype(np.uint32)
    hdr[:, 1] = (t % np.uint64(1000000)).astype(np.uint32)
    hdr[:, 2] = size
    hdr[:, 3] = size
    r[:, :16] = hdr.view(np.uint8).reshape(n, 16)
    r[:, 16:] = frames
    return r


def pcap_fixed(n, size=64, seed=1, ipv6=False, proto=17, vlan=None, fcs=False):
    """n records of `size`-byte IPv4/UDP (or IPv6, TCP) frames; vlan=TCI tags them,
    fcs appends a 4-byte FCS (as pcap_imix)."""
    rng = np.random.default_rng(seed)
    recs = _records(_frames(rng, n, size, ipv6=ipv6, proto=proto), 0)
    if vlan is not None:
        recs = _tag(recs, vlan)
    if fcs:
        recs = _fcs(recs, rng)
    return PCAP_HDR.tobytes() + recs.tobytes()


def _tag(recs, tci):
    """(n, 16 + size) records -> (n, 20 + size): an 802.1Q tag {0x8100, tci} after the MACs"""
    n, w = recs.shape
    out = np.empty((n, w + 4), np.uint8)
    out[:, :28] = recs[:, :28]
    out[:, 28:32] = (0x81, 0x00, (tci >> 8) & 0xFF, tci & 0xFF)
    out[:, 32:] = recs[:, 28:]
    hdr = out[:, :16].copy().view("<u4")
    hdr[:, 2] += 4
    hdr[:, 3] += 4
    out[:, :16] = hdr.view(np.uint8)
    return out


def _fcs(recs, rng):
    """(n, 16 + size) records -> (n, 20 + size): 4 trailing frame-check bytes (random
    values: no edit reads them, --efcs strips them) counted in caplen and len"""
    n, w = recs.shape
    out = np.empty((n, w + 4), np.uint8)
    out[:, :w] = recs
    out[:, w:] = rng.integers(0, 256, size=(n, 4), dtype=np.uint8)
    hdr = out[:, :16].copy().view("<u4")
    hdr[:, 2] += 4
    hdr[:, 3] += 4
    out[:, :16] = hdr.view(np.uint8)
    return out


def pcap_imix(n, seed=1, chunk=1 << 20, vlan=None, fcs=False):
    """n records cycling 64x7, 570x4, 1514x1 (deterministic 7:4:1); vlan=TCI: every
    frame carries an 802.1Q tag (68/574/1518 bytes); fcs: every frame ends in a 4-byte
    FCS (the IP lengths exclude it, as on a capture taken with FCS)."""
    rng = np.random.default_rng(seed)
    pat = IMIX_PATTERN
    grow = (4 if vlan is not None else 0) + (4 if fcs else 0)
    cyc_len = sum(16 + s + grow for s in pat)
    parts = [PCAP_HDR.tobytes()]
    done = 0
    while done < n:
        m = min(chunk, n - done)
        ncyc = (m + len(pat) - 1) // len(pat)
        buf = np.empty((ncyc, cyc_len), np.uint8)
        off = 0
        counts = {s: pat.count(s) for s in set(pat)}
        made = {s: _records(_frames(rng, ncyc * counts[s], s, first_index=done), done) for s in counts}
        if vlan is not None:
            made = {s: _tag(r, vlan) for s, r in made.items()}
        if fcs:
            made = {s: _fcs(r, rng) for s, r in made.items()}
        used = {s: 0 for s in counts}
        for s in pat:
            rec = made[s][used[s]::counts[s]]
            used[s] += 1
            buf[:, off:off + 16 + s + grow] = rec
            off += 16 + s + grow
        flat = buf.reshape(-1)
        if ncyc * len(pat) != m:  # trim the last partial cycle
            keep = m - (ncyc - 1) * len(pat)
            end = (ncyc - 1) * cyc_len + sum(16 + s + grow for s in pat[:keep])
            flat = flat[:end]
        parts.append(flat.tobytes())
        done += m
    return b"".join(parts)


def pcap_mixed_v4v6(n, size=1514, seed=1):
    """n records of `size` bytes, alternating IPv4/IPv6 and UDP/TCP (config 5)."""
    rng = np.random.default_rng(seed)
    quarter = (n + 3) // 4
    kinds = [(False, 17), (True, 17), (False, 6), (True, 6)]
    made = [_records(_frames(rng, quarter, size, ipv6=v6, proto=p), 0) for v6, p in kinds]
    recs = np.empty((quarter * 4, 16 + size), np.uint8)
    for k in range(4):
        recs[k::4] = made[k]
    recs = recs[:n]
    hdr = recs[:, :16].copy().view("<u4")
    t = np.arange(n, dtype=np.uint32)
    hdr[:, 0] = 1600000000
    hdr[:, 1] = t
    recs[:, :16] = hdr.view(np.uint8)
    return PCAP_HDR.tobytes() + recs.tobytes()


def tcpprep_cache(n, seed=1, nosend_every=0):
    """tcpprep v04 cache (cache.h:63-72): 2 bits per packet, 4 packets per byte.

    Direction alternates C2S/S2C in runs of 1-3 packets ("by flow"); with
    nosend_every=k every k-th packet is NOSEND."""
    rng = np.random.default_rng(seed)
    runs = rng.integers(1, 4, n)
    d = (np.cumsum(runs)[:n] & 1).astype(np.uint8)  # 1 -> C2S, 0 -> S2C
    d = np.repeat(d, 1)[:n]
    send = np.ones(n, np.uint8)
    if nosend_every:
        send[nosend_every - 1::nosend_every] = 0
    bits = (send << 1) | d  # bit 2k+1 = send, bit 2k = C2S
    pad = (-n) % 4
    b = np.concatenate([bits, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    data = (b[:, 0] | (b[:, 1] << 2) | (b[:, 2] << 4) | (b[:, 3] << 6)).astype(np.uint8)
    comment = b"synthetic"
    hdr = b"tcpprep\x00" + b"04\x00\x00" + int(n).to_bytes(8, "big") + (4).to_bytes(2, "big") + \
        len(comment).to_bytes(2, "big")
    return hdr + comment + data.tobytes()


def records(pcap: bytes):
    """split a little-endian pcap image into (ts_sec, ts_usec, caplen, len, data) tuples."""
    out = []
    off = 24
    while off + 16 <= len(pcap):
        ts, tu, cl, ln = np.frombuffer(pcap[off:off + 16], "<u4")
        out.append((int(ts), int(tu), int(cl), int(ln), pcap[off + 16:off + 16 + int(cl)]))
        off += 16 + int(cl)
    return out


def build_pcap(recs, linktype=1):
    """(ts_sec, ts_usec, caplen, len, data) tuples -> pcap image."""
    hdr = bytearray(PCAP_HDR.tobytes())
    hdr[20:24] = int(linktype).to_bytes(4, "little")
    parts = [bytes(hdr)]
    for ts, tu, cl, ln, data in recs:
        parts.append(np.array([ts, tu, cl, ln], "<u4").tobytes() + bytes(data[:cl]))
    return b"".join(parts)


# link types of the non-Ethernet decoders (the pcap header's linktype field)
LINKTYPES = {"sll": 113, "sll2": 276, "raw": 101, "raw12": 12, "null": 0, "loop": 108, "ppp": 50, "chdlc": 104}
# ... and of the Juniper Ethernet, 802.11 and radiotap decoders
LINKTYPES_MORE = {"jnpr": 178, "80211": 105, "radiotap": 127}


def _jnpr(i, d, odd, rng):
    """a Juniper Ethernet header {4d 47 43, options (L2 present | direction), extension
    length} with TLV extensions (an ifindex TLV first on some records), media type 1 and
    encapsulation 14, then the whole Ethernet frame; every 4th inner frame carries an
    802.1Q tag.  odd: a bad magic (a decoder error)."""
    ext = b""
    if i % 3 == 1:
        ext += b"\x01\x04" + int(i).to_bytes(4, "big")
    ext += (b"\x06\x01\x0e\x03\x01\x01" if i % 2 else b"\x03\x01\x01\x06\x01\x0e")
    if i % 5 == 2:
        ext += b"\x04\x02\x00\x07"  # a TLV after both (the walk has stopped)
    magic = b"\x4d\x47\x44" if odd else b"\x4d\x47\x43"
    h = magic + bytes([0x80 | (i & 1)]) + len(ext).to_bytes(2, "big") + ext
    if i % 4 == 3:
        d = d[:12] + b"\x81\x00" + int(0x2000 | (i % 4095)).to_bytes(2, "big") + d[12:]
    return h + d


def _w80211(i, d, odd, rng):
    """an 802.11 data frame: frame control (data, or QoS data on every 3rd record; the
    DS bits cycle 0..3, four addresses for ToDS|FromDS), duration, addresses, sequence,
    [QoS control], an 802.2 SNAP header with the ethertype, then the L3 bytes.  odd: a
    management frame, a protected frame or an 802.2 header without SNAP, in turn."""
    ds = i % 4
    qos = i % 3 == 0
    b0 = 0x88 if qos else 0x08
    b1 = ds
    llc = b"\xaa\xaa\x03\x00\x00\x00" + d[12:14]
    if odd:
        k = (i // 7) % 3
        if k == 0:
            b0 = 0x80  # a beacon: not a data frame
        elif k == 1:
            b1 |= 0x40  # protected
        else:
            llc = b"\x42\x42\x03" + bytes(5)
    a = [d[0:6], d[6:12], bytes(rng.integers(0, 256, 6, dtype=np.uint8)), bytes(rng.integers(0, 256, 6, dtype=np.uint8))]
    hdr = bytes([b0, b1]) + b"\x2c\x00" + a[0] + a[1] + a[2] + (i % 4096 * 16).to_bytes(2, "little")
    if ds == 3:
        hdr += a[3]
    if qos:
        hdr += bytes([i % 8, 0])
    return hdr + llc + d[14:]


def _radiotap(i, d, odd, rng):
    """a radiotap header (version 0, length 8 + 4 k, present flags) before an 802.11 frame"""
    extra = 4 * (i % 3)
    rt = b"\x00\x00" + (8 + extra).to_bytes(2, "little") + (0x0000002e).to_bytes(4, "little") + bytes(extra)
    return rt + _w80211(i, d, odd, rng)


def reframe(pcap: bytes, kind: str, seed=1, odd_every=0):
    """An Ethernet II capture re-framed for another DLT: the 14-byte Ethernet header is
    replaced by the link's own header (the L3 bytes, timestamps and the caplen/len
    difference are kept):
      sll    Linux cooked v1 (16 B): packet type, ARPHRD_ETHER, address length 6, the
             source MAC (+2 pad), the ethertype
      sll2   Linux cooked v2 (20 B): ethertype, reserved, ifindex, ARPHRD_ETHER, packet
             type, address length, source MAC (+2 pad)
      raw / raw12  no header (linktype 101 / 12)
      null   the address family in host (little-endian) order: 2 or, for IPv6, one of the
             four values the reference takes (10, 24, 28, 30)
      loop   the address family in network order
      ppp    PPP in HDLC-like framing: ff 03 and the PPP protocol (0x0021 IPv4, 0x0057 IPv6)
      chdlc  Cisco HDLC: address 0x0f, control 0, the ethertype
      jnpr / 80211 / radiotap  see _jnpr, _w80211, _radiotap (the whole frame is kept or
             rebuilt around the L3 bytes)
    odd_every=k: every k-th record gets a header the decoder refuses or does not take as
    IP (SLL: ARPHRD 0x0200; NULL/LOOP: family 7; PPP: protocol 0xc021; RAW: version 5)."""
    rng = np.random.default_rng(seed)
    out = []
    for i, (ts, tu, cl, ln, d) in enumerate(records(pcap)):
        if cl < 14:
            out.append((ts, tu, cl, ln, d))
            continue
        et, dmac, smac, l3 = d[12:14], d[0:6], d[6:12], d[14:]
        v6 = et == b"\x86\xdd"
        odd = odd_every and i % odd_every == odd_every - 1
        if kind == "sll":
            h = bytes([0, int(rng.integers(0, 5))]) + (b"\x02\x00" if odd else
                                                          (b"\x00\x01" if i % 3 else b"\x03\x04")) + \
                b"\x00\x06" + smac + b"\x00\x00" + et
        elif kind == "sll2":
            h = et + b"\x00\x00" + int(i % 7 + 1).to_bytes(4, "big") + (b"\x02\x00" if odd else b"\x00\x01") + \
                bytes([int(rng.integers(0, 5)), 6]) + smac + b"\x00\x00"
        elif kind in ("raw", "raw12"):
            h = b""
            if odd:
                l3 = bytes([0x50 | (l3[0] & 15)]) + l3[1:]
        elif kind in ("null", "loop"):
            af = 7 if odd else ([10, 24, 28, 30][i % 4] if v6 else 2)
            h = af.to_bytes(4, "big" if kind == "loop" else "little")
        elif kind == "ppp":
            h = b"\xff\x03" + (b"\xc0\x21" if odd else (b"\x00\x57" if v6 else b"\x00\x21"))
        elif kind == "chdlc":
            h = b"\x0f\x00" + et
        elif kind in LINKTYPES_MORE:
            nd = {"jnpr": _jnpr, "80211": _w80211, "radiotap": _radiotap}[kind](i, d, odd, rng)
            dl = len(nd) - len(d)
            out.append((ts, tu, cl + dl, ln + dl, nd))
            continue
        else:
            raise ValueError(kind)
        nd = h + l3
        dl = len(nd) - len(d)
        out.append((ts, tu, cl + dl, ln + dl, nd))
    return build_pcap(out, {**LINKTYPES, **LINKTYPES_MORE}[kind])
