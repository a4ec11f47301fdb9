"""Synthetic captures for the fast-lane tests: the header shapes the register-
resident lane carries (Ethernet II + IPv4 IHL 5 / IPv6, TCP/UDP, caplen == len,
consistent lengths) mixed with near misses it must hand to the generic lane
(VLAN tags, IP options, fragments, caplen < len, Ethernet padding, IPv6
extension headers, ICMP, ARP, odd lengths, jumbo and >16 KiB records).
Checksums are valid unless a case wants otherwise."""
import random
import struct

from tcpreplay_amd import synth as S


def csum(data: bytes) -> int:
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def mac(rng, kind="uni"):
    if kind == "bcast":
        return b"\xff" * 6
    if kind == "mcast4":
        return bytes([1, 0, 0x5E, rng.randrange(128), rng.randrange(256), rng.randrange(256)])
    if kind == "mcast6":
        return bytes([0x33, 0x33]) + bytes(rng.randrange(256) for _ in range(4))
    if kind == "vrrp":
        return bytes([0, 0, 0x50, 0, rng.choice([1, 2]), rng.randrange(256)])
    return bytes([rng.randrange(256) & 0xFE]) + bytes(rng.randrange(256) for _ in range(5))


def l4(rng, proto, src_ph: bytes, paylen, udp_zero=False, tcp_opts=0):
    sport, dport = rng.choice([53, 80, 443, 8080, rng.randrange(1, 65536)]), rng.choice(
        [53, 80, 443, 5353, rng.randrange(1, 65536)])
    payload = bytes(rng.randrange(256) for _ in range(paylen))
    if proto == 17:
        ln = 8 + paylen
        h = struct.pack("!HHHH", sport, dport, ln, 0)
        c = csum(src_ph + struct.pack("!BBH", 0, 17, ln) + h + payload)
        if udp_zero:
            c = 0
        elif c == 0:
            c = 0xFFFF
        return h[:6] + struct.pack("!H", c) + payload
    opts = bytes(rng.randrange(256) for _ in range(4 * tcp_opts))
    doff = 5 + tcp_opts
    h = struct.pack("!HHIIBBHHH", sport, dport, rng.randrange(1 << 32), rng.randrange(1 << 32), doff << 4,
                    rng.choice([0x18, 0x10, 0x02, 0x12]), 65535, 0, 0) + opts
    seg = h + payload
    c = csum(src_ph + struct.pack("!BBH", 0, 6, len(seg)) + seg)
    return seg[:16] + struct.pack("!H", c) + seg[18:]


def ipv4_pkt(rng, proto, paylen, dst_kind="uni", udp_zero=False, opts=0, frag=0, tcp_opts=0):
    src = bytes([10, rng.randrange(256), rng.randrange(256), rng.randrange(1, 255)])
    if dst_kind == "mcast":
        dst = bytes([224 + rng.randrange(16), rng.randrange(256), rng.randrange(256), rng.randrange(256)])
    elif dst_kind == "bcast":
        dst = b"\xff\xff\xff\xff"
    else:
        dst = bytes([rng.choice([172, 192, 10, 8]), rng.randrange(256), rng.randrange(256), rng.randrange(1, 255)])
    seg = l4(rng, proto, src + dst, paylen, udp_zero, tcp_opts)
    ihl = 5 + opts
    optb = bytes(rng.randrange(256) for _ in range(4 * opts))
    tot = 4 * ihl + len(seg)
    h = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, rng.randrange(256), tot, rng.randrange(65536), frag,
                    rng.randrange(1, 256), proto, 0, src, dst) + optb
    h = h[:10] + struct.pack("!H", csum(h)) + h[12:]
    return h + seg


def ipv6_pkt(rng, proto, paylen, dst_kind="uni", udp_zero=False, ext=False):
    src = bytes([0x20, 0x01]) + bytes(rng.randrange(256) for _ in range(14))
    if dst_kind == "mcast":
        dst = b"\xff\x02" + bytes(rng.randrange(256) for _ in range(14))
    else:
        dst = bytes([0x26, 0x06]) + bytes(rng.randrange(256) for _ in range(14))
    seg = l4(rng, proto, src + dst, paylen, udp_zero)
    nh = proto
    if ext:  # hop-by-hop header in front
        seg = bytes([proto, 0]) + bytes(6) + seg
        nh = 0
    h = struct.pack("!IHBB16s16s", (6 << 28) | (rng.randrange(256) << 20) | rng.randrange(1 << 20), len(seg), nh,
                    rng.randrange(1, 256), src, dst)
    return h + seg


def frame(rng, l3: bytes, et, dst_kind="uni", vlan=False, pad=0):
    f = mac(rng, dst_kind) + mac(rng)
    if vlan:
        f += struct.pack("!HH", 0x8100, rng.randrange(65536))
    return f + struct.pack("!H", et) + l3 + bytes(pad)


def mixed(n, seed, near_miss=0.25, max_pay=1460):
    """n records; roughly 1-near_miss of them fast-lane shapes."""
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        r = rng.random()
        proto = rng.choice([6, 17])
        size_pick = rng.random()
        if size_pick < 0.4:
            paylen = rng.randrange(0, 40)
        elif size_pick < 0.8:
            paylen = rng.randrange(0, max_pay)
        else:
            paylen = rng.choice([18, 22, 26, 480, 536, 1460, 1472])
        caplen_cut = None
        length_extra = 0
        if r >= near_miss:
            kind = rng.random()
            dk = rng.choice(["uni"] * 6 + ["mcast", "bcast"])
            if kind < 0.55:
                l3 = ipv4_pkt(rng, proto, paylen, dst_kind=dk, udp_zero=rng.random() < 0.05)
                et = 0x0800
            else:
                if near_miss == 0.0 and ((paylen + (8 if proto == 17 else 20)) & 0xFF) == 0:
                    paylen += 1  # keep clear of the raw network-order length compare (edit_packet.c:167)
                l3 = ipv6_pkt(rng, proto, paylen, dst_kind="mcast" if dk == "mcast" else "uni",
                              udp_zero=rng.random() < 0.05)
                et = 0x86DD
            mk = rng.choice(["uni"] * 8 + ["bcast", "mcast4", "mcast6", "vrrp"])
            f = frame(rng, l3, et, dst_kind=mk)
        else:
            miss = rng.randrange(9)
            if miss == 0:
                f = frame(rng, ipv4_pkt(rng, proto, paylen), 0x0800, vlan=True)
            elif miss == 1:
                f = frame(rng, ipv4_pkt(rng, proto, paylen, opts=rng.randrange(1, 4)), 0x0800)
            elif miss == 2:
                f = frame(rng, ipv4_pkt(rng, 17, paylen, frag=rng.choice([0x2000, 0x0010])), 0x0800)
            elif miss == 3:  # Ethernet padding after a short IP datagram
                f = frame(rng, ipv4_pkt(rng, 17, rng.randrange(0, 10)), 0x0800, pad=rng.randrange(1, 20))
            elif miss == 4:
                f = frame(rng, ipv6_pkt(rng, proto, paylen, ext=True), 0x86DD)
            elif miss == 5:  # ICMP
                f = frame(rng, ipv4_pkt(rng, 1, paylen), 0x0800)
            elif miss == 6:  # ARP
                f = frame(rng, bytes([0, 1, 8, 0, 6, 4, 0, 1]) + bytes(rng.randrange(256) for _ in range(20)),
                          0x0806)
            elif miss == 7:  # snaplen-truncated capture
                f = frame(rng, ipv4_pkt(rng, proto, paylen + 40), 0x0800)
                caplen_cut = rng.randrange(14, len(f))
            else:  # len != caplen
                f = frame(rng, ipv6_pkt(rng, proto, paylen), 0x86DD)
                length_extra = rng.randrange(1, 60)
        data = f if caplen_cut is None else f[:caplen_cut]
        recs.append((1600000000 + i // 1000, i % 1000000, len(data), len(f) + length_extra, data))
    return recs


def build(recs):
    return S.build_pcap(recs)
