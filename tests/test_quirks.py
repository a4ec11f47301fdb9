"""The reference's bug-compatible behaviours, pinned to the bytes
the survey observed running the reference code, not only to the oracle.

Each case is a hand-built capture, the option line, and a check of literal output bytes:
  Q3  multicast IPv4 dst -> dst MAC 01:00:5e:01:02:03, with no options and with
      --enet-dmac (en10mb.c:867-884)
  Q4  a 60-byte padded frame (ip_len 28, header checksum 0xbeef) is written unchanged by
      --fixcsum (edit_packet.c:84-92)
  Q5  a UDP checksum that computes to 0 is written 00 00 (checksum.c:125, checksum.h:25)
  Q6  IPv6 -> fragment header -> UDP: checksummed as TCP, i.e. the two bytes at L4+16 are
      overwritten (get_ipv6_l4proto returns 44, checksum.c:80-81)
  Q9  test.pcap packet 29 under --pnat=[::/0]:[2001:db8:aaaa::/36]: src 2001:db8:15a0:...,
      dst 1:db8::... (remap_ipv6's stray write, edit_packet.c:772-776)
  Q11 --enet-vlan=add --enet-vlan-tag=7 on a TCI 0xb02d frame pushes a second tag:
      81 00 b0 07 81 00 b0 2d (en10mb.c:526-529,696-703)
  Q12 an IPv4 version-5 header in packet 3 of 4 aborts the run with 2 packets written
      (edit_packet.c:73-79, tcprewrite.c:156-160)
The CPU tests check the oracle against these bytes; the GPU tests check the device path
against the same bytes and the oracle.
"""
import struct

import pytest

import golden_cases as G
import oracle_lib as O
from tcpreplay_amd import synth as S


def _csum(data: bytes) -> int:
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack(f">{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _ipv4_udp(dst=b"\xac\x10\x01\x02", payload=b"\x11" * 22, udp_sum=None, vlan=None):
    """Ethernet/IPv4/UDP frame with valid checksums (or udp_sum as given)"""
    udp_len = 8 + len(payload)
    ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + udp_len, 1, 0, 64, 17, 0, b"\x0a\x00\x00\x01", dst))
    struct.pack_into(">H", ip, 10, (~_csum(bytes(ip))) & 0xFFFF)
    udp = bytearray(struct.pack(">HHHH", 1234, 53, udp_len, 0) + payload)
    if udp_sum is None:
        c = (~_csum(bytes(ip[12:20]) + struct.pack(">HH", 17, udp_len) + bytes(udp))) & 0xFFFF
        udp_sum = c or 0xFFFF
    struct.pack_into(">H", udp, 6, udp_sum)
    l2 = bytes.fromhex("001122334455" "00667788 99aa".replace(" ", ""))
    if vlan is not None:
        l2 += b"\x81\x00" + struct.pack(">H", vlan)
    return l2 + b"\x08\x00" + bytes(ip) + bytes(udp)


def _pcap(frames):
    return S.build_pcap([(1, i, len(f), len(f), f) for i, f in enumerate(frames)])


def _q3():
    f = _ipv4_udp(dst=bytes([239, 1, 2, 3]))
    return _pcap([f]), 0, 0, 6, bytes.fromhex("01005e010203")


def _q4_frame():
    f = bytearray(_ipv4_udp(payload=b""))  # ip_len 28
    struct.pack_into(">H", f, 24, 0xBEEF)
    return bytes(f) + bytes(60 - len(f))


def _q5_frame():
    """a UDP packet whose checksum sum folds to 0xffff: one payload word is chosen so"""
    base = bytearray(_ipv4_udp(payload=bytes(20) + b"\0\0"))
    ip, udp = base[14:34], bytearray(base[34:])
    struct.pack_into(">H", udp, 6, 0)
    pseudo = bytes(ip[12:20]) + struct.pack(">HH", 17, len(udp))
    for w in range(65536):
        struct.pack_into(">H", udp, len(udp) - 2, w)
        if _csum(pseudo + bytes(udp)) == 0xFFFF:
            break
    struct.pack_into(">H", udp, 6, 0x1234)  # non-zero: the reference recomputes it
    return bytes(base[:34]) + bytes(udp)


def _q6_frame():
    payload = bytes(range(40))
    udp = struct.pack(">HHHH", 1000, 2000, 8 + len(payload), 0x4321) + payload
    frag = struct.pack(">BBHI", 17, 0, 0, 0x01020304)  # next header UDP, offset 0, M=0
    src = bytes.fromhex("20010db8000000000000000000000001")
    dst = bytes.fromhex("20010db8000000000000000000000002")
    ip6 = struct.pack(">IHBB", 0x60000000, len(frag) + len(udp), 44, 64) + src + dst
    return bytes.fromhex("001122334455006677889 9aa".replace(" ", "")) + b"\x86\xdd" + ip6 + frag + udp


def _q6_expect(frame):
    """do_checksum's TCP case over the UDP header + payload: pseudo header of the
    L4 length and IPPROTO_TCP, the sum field at L4+16"""
    l4 = bytearray(frame[62:])
    l4[16:18] = b"\0\0"
    s = _csum(frame[22:54] + struct.pack(">HH", 6, len(l4)) + bytes(l4))
    return ((~s) & 0xFFFF).to_bytes(2, "big")


def _q12_pcap():
    recs = S.records(G.read("test.pcap"))[:4]
    ts, tu, cl, ln, d = recs[2]
    d = bytearray(d)
    assert d[12:14] == b"\x08\x00"
    d[14] = 0x55
    recs[2] = (ts, tu, cl, ln, bytes(d))
    return S.build_pcap(recs)


def check_q3(rewrite):
    pcap, *_ = _q3()
    for args in ([], ["--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66"], ["--fixcsum"]):
        rc, out = rewrite(pcap, args)
        assert rc == 0
        assert S.records(out)[0][4][0:6] == bytes.fromhex("01005e010203"), args


def check_q4(rewrite):
    f = _q4_frame()
    pcap = _pcap([f])
    rc, out = rewrite(pcap, ["--fixcsum"])
    assert rc == 0 and S.records(out)[0][4] == f


def check_q5(rewrite):
    f = _q5_frame()
    rc, out = rewrite(_pcap([f]), ["--fixcsum"])
    assert rc == 0
    o = S.records(out)[0][4]
    assert o[40:42] == b"\x00\x00" and o[24:26] == f[24:26] and o[:40] == f[:40] and o[42:] == f[42:]


def check_q6(rewrite):
    f = _q6_frame()
    rc, out = rewrite(_pcap([f]), ["--fixcsum"])
    assert rc == 0
    o = S.records(out)[0][4]
    assert o[78:80] == _q6_expect(f) != f[78:80]
    assert o[:78] == f[:78] and o[80:] == f[80:]  # the UDP checksum field (L4+6) is untouched


def check_q9(rewrite):
    rc, out = rewrite(G.read("test.pcap"), ["--pnat=[::/0]:[2001:db8:aaaa::/36]"])
    assert rc == 0
    p29 = S.records(out)[28][4]
    assert p29[12:14] == b"\x86\xdd"
    assert p29[22:28] == bytes.fromhex("20010db815a0")  # src 2001:db8:15a0:...  (/36 nibble not applied)
    assert p29[38:54] == bytes.fromhex("00010db800000000000000006812069c")  # dst 2606:4700:: -> 1:db8::


def check_q11(rewrite):
    f = _ipv4_udp(vlan=0xB02D)
    rc, out = rewrite(_pcap([f]), ["--enet-vlan=add", "--enet-vlan-tag=7"])
    assert rc == 0
    o = S.records(out)[0]
    assert o[4][12:20] == bytes.fromhex("8100b0078100b02d") and o[2] == len(f) + 4


def check_q12(rewrite):
    rc, out = rewrite(_q12_pcap(), ["--fixcsum"])
    assert rc == -1 and len(S.records(out)) == 2


CHECKS = [check_q3, check_q4, check_q5, check_q6, check_q9, check_q11, check_q12]


@pytest.mark.parametrize("check", CHECKS, ids=[c.__name__[6:] for c in CHECKS])
def test_oracle_reproduces_reference_quirk(built, check):
    check(O.rewrite)


@pytest.mark.gpu
@pytest.mark.parametrize("check", CHECKS, ids=[c.__name__[6:] for c in CHECKS])
def test_gpu_reproduces_reference_quirk(built, check):
    import tcpreplay_amd as TA

    def gpu(pcap, args):
        te = TA.TcpEdit(args)
        try:
            rc, out = te.rewrite(pcap)
        finally:
            te.close()
        rc_o, exp = O.rewrite(pcap, args)
        assert rc == rc_o and out == exp
        return rc, out

    check(gpu)


def test_hdlc_encoder_falls_back_on_the_decoded_vlan_flag(built):
    """--dlt=hdlc without --hdlc-address/--hdlc-control on Ethernet: dlt_hdlc_encode reads
    `extra->hdlc`, the first int of the decoded extra -- the en10mb decoder's `vlan` flag
    (en10mb_types.h:30): a tagged frame gets address = control = 1 and the proto, an untagged
    one fails after the memmove of its payload to byte 4 (hdlc.c:240-288) and is written as
    that left it (a soft error, caplen unchanged).  Parity unpinned: no reference fixture."""
    import tcpreplay_amd.synth as S
    base = S.records(S.pcap_fixed(6, 90, seed=4))
    recs = []
    for i, (ts, tu, cl, ln, d) in enumerate(base):
        if i % 2:
            d = d[:12] + b"\x81\x00\x20\x05" + d[12:]
            cl, ln = cl + 4, ln + 4
        recs.append((ts, tu, cl, ln, d))
    rc, out = O.rewrite(S.build_pcap(recs), ["--dlt=hdlc"])
    assert rc == 0
    for i, (r_in, r_out) in enumerate(zip(recs, S.records(out))):
        d = r_in[4]
        if i % 2:  # {1, 1, ctx->proto}: the outer type, 0x8100 (en10mb.c:431) + the L3 bytes
            assert r_out[4] == b"\x01\x01\x81\x00" + d[18:] and r_out[2] == r_in[2] - 14
        else:      # d[0:4] + the payload moved to byte 4 + the last 10 bytes as they were
            assert r_out[2:4] == r_in[2:4] and r_out[4] == d[:4] + d[14:] + d[-10:]
