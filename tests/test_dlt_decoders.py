"""The non-Ethernet decoders: DLT_LINUX_SLL, LINUX_SLL2, RAW, NULL,
LOOP, PPP_SERIAL and C_HDLC input (src/tcpedit/plugins/dlt_{linuxsll,linuxsll2,raw,null,
loop,pppserial,hdlc}), into their own plugins as encoders (which refuse to encode, or for
pppserial pass the packet through), into the en10mb encoder (--dlt=enet: a 14-byte
Ethernet header replaces the decoded one), and into the user and hdlc encoders.

Parity is unpinned: the reference ships no capture of these link types.  The oracle's
restatement (oracle/tcpedit_oracle.c decoder_proto/decoder_decode and the en10mb
encoder's other-DLT branch) is checked here against outputs built independently from
the re-framed captures (CPU), and the GPU against the oracle (bit-exact), including the
Q18 carry of the en10mb encoder's dst_modified across S2C records behind a Linux cooked
decoder."""
import struct

import pytest

import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

KINDS = list(S.LINKTYPES)
DLT_OF = {"sll": 113, "sll2": 276, "raw": 12, "raw12": 12, "null": 0, "loop": 108, "ppp": 50, "chdlc": 104}
MACS = ["--enet-smac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee", "--enet-dmac=00:66:77:88:99:aa,00:12:34:56:78:9a"]


def _base(n=600, seed=3):
    return S.pcap_imix(n, seed=seed)


def _eth_of(kind, rec_in, dmac, smac):
    """the --dlt=enet output record of one re-framed record, built from its layout (None:
    the decoder refuses it or does not take it as IP, so it is written unchanged)"""
    ts, tu, cl, ln, d = rec_in
    hl = {"sll": 16, "sll2": 20, "raw": 0, "raw12": 0, "null": 4, "loop": 4, "ppp": 4, "chdlc": 4}[kind]
    if kind == "sll":
        ok, et = d[2:4] in (b"\x00\x01", b"\x03\x04"), d[14:16]
    elif kind == "sll2":
        ok, et = d[8:10] == b"\x00\x01", d[0:2]
    elif kind in ("raw", "raw12"):
        ok, et = d[0] >> 4 in (4, 6), (b"\x08\x00" if d[0] >> 4 == 4 else b"\x86\xdd")
    elif kind in ("null", "loop"):
        af = int.from_bytes(d[0:4], "big" if kind == "loop" else "little")
        ok, et = af in (2, 10, 24, 28, 30), (b"\x08\x00" if af == 2 else b"\x86\xdd")
    elif kind == "ppp":  # pppserial takes only its IPv4 protocol (0x0021), and never as IP
        ok, et = d[2:4] == b"\x00\x21", b"\x08\x00"
    else:
        ok, et = True, d[2:4]
    if not ok:
        return None
    out = dmac + smac + et + d[hl:]
    dl = len(out) - len(d)
    return (ts, tu, cl + dl, ln + dl, out)


@pytest.mark.parametrize("kind", KINDS)
def test_oracle_own_encoder_writes_the_capture_unedited(built, kind):
    """no --dlt: the decoder's own plugin encodes -- linuxsll/linuxsll2/raw/null/loop refuse
    (every packet a soft error, written as read), pppserial passes it through, hdlc needs
    its two options; the output header carries the link type (DLT_RAW as LINKTYPE_RAW)"""
    pcap = S.reframe(_base(), kind, odd_every=7)
    rc, out = O.rewrite(pcap, ["--fixcsum", "--seed=7", "--pnat=10.0.0.0/8:192.168.0.0/16"])
    assert rc == 0
    assert S.records(out) == S.records(pcap)
    assert struct.unpack_from("<I", out, 20)[0] == (101 if kind.startswith("raw") else S.LINKTYPES[kind])
    rc, out = O.rewrite(pcap, ["--fixcsum", "--skip-soft-errors"])
    assert rc == 0
    # pppserial's proto takes only its IPv4 protocol: the rest are soft errors, dropped here
    kept = [r for r in S.records(pcap) if r[4][2:4] == b"\x00\x21"] if kind == "ppp" else []
    assert S.records(out) == kept


@pytest.mark.parametrize("kind", KINDS)
def test_oracle_into_ethernet_matches_the_layout(built, kind):
    """--dlt=enet with both MACs and no other edit: each record becomes the given MACs,
    the decoded ethertype and its L3 bytes; records the decoder refuses stay as read"""
    pcap = S.reframe(_base(), kind, odd_every=7)
    rc, out = O.rewrite(pcap, ["--dlt=enet"] + MACS)
    assert rc == 0
    assert struct.unpack_from("<I", out, 20)[0] == 1
    dmac, smac = bytes.fromhex("00667788 99aa".replace(" ", "")), bytes.fromhex("001122334455")
    exp = [_eth_of(kind, r, dmac, smac) or r for r in S.records(pcap)]
    assert S.records(out) == exp


def test_oracle_cooked_source_address_and_zero_destination(built):
    """a Linux cooked decoder has Ethernet addresses (linuxsll.c:186-188): without
    --enet-smac the source is the cooked header's address; the destination the context
    never set is zero"""
    pcap = S.reframe(_base(50), "sll")
    rc, out = O.rewrite(pcap, ["--dlt=enet"])
    assert rc == 0
    for r_in, r_out in zip(S.records(pcap), S.records(out)):
        assert r_out[4][:6] == bytes(6) and r_out[4][6:12] == r_in[4][6:12] and r_out[4][14:] == r_in[4][16:]


def test_unserved_combinations_are_refused(built):
    te = TA.TcpEdit
    for dlt, args in [(1, ["--dlt=tokenring"])]:
        with pytest.raises(Exception):
            te(args, dlt=dlt)
    with pytest.raises(Exception):
        te(["--fixcsum"], dlt=9)  # DLT_PPP: the reference has no plugin for it either


@pytest.mark.parametrize("kind", ["raw", "null", "ppp", "chdlc"])
def test_oracle_failing_encodes_write_the_half_moved_record(built, kind):
    """decoders without Ethernet addresses: --dlt=enet without --enet-dmac fails every packet
    after the encoder's memmove of the payload from the decoded l2len to byte 14 (en10mb.c:
    567-578) and after the source address (:586-619); --dlt=hdlc without its fields after the
    memmove to byte 4 (hdlc.c:240-288).  The soft error writes the record as that left it,
    its caplen unchanged (tcpedit.c:104-108); a record the decoder refuses is written as read"""
    pcap = S.reframe(_base(300, seed=31), kind, odd_every=7)
    hl = {"raw": 0, "null": 4, "ppp": 4, "chdlc": 4}[kind]
    smac = bytes.fromhex("001122334455")
    rc, out = O.rewrite(pcap, ["--dlt=enet", "--enet-smac=00:11:22:33:44:55"])
    assert rc == 0
    for r_in, r_out in zip(S.records(pcap), S.records(out)):
        d, o = r_in[4], r_out[4]
        assert r_out[2:4] == r_in[2:4]
        if _eth_of(kind, r_in, b"", b"") is None:  # (the decoder's soft error: as read)
            assert o == d
            continue
        moved = bytearray(d) + bytes(14 - hl)
        moved[14:14 + len(d) - hl] = d[hl:]
        moved[6:12] = smac
        assert o == bytes(moved[:len(d)])
    rc, out = O.rewrite(pcap, ["--dlt=hdlc", "--hdlc-address=9"])
    assert rc == 0
    for r_in, r_out in zip(S.records(pcap), S.records(out)):
        d, o = r_in[4], r_out[4]
        if _eth_of(kind, r_in, b"", b"") is None:
            assert o == d
            continue
        moved = bytearray(d) + bytes(4)
        moved[4:4 + len(d) - hl] = d[hl:]
        moved[0] = 9  # the address goes in before the control field fails
        assert r_out[2:4] == r_in[2:4] and o == bytes(moved[:len(d)])


@pytest.mark.parametrize("kind", ["raw", "sll"])
def test_oracle_vlan_push_behind_another_decoder(built, kind):
    """--enet-vlan=add with both MACs: an 18-byte header from 14 + 4 (en10mb.c:547), the TCI at
    the decoder extra's never-set vlan_offset 0 over the destination address, the inner type
    the context's never-set proto_vlan_tag 0 (:696-715), bytes [14, 18) the packet's own"""
    pcap = S.reframe(_base(200, seed=33), kind, odd_every=9)
    hl = {"raw": 0, "sll": 16}[kind]
    rc, out = O.rewrite(pcap, ["--dlt=enet", "--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-pri=5"] + MACS)
    for r_in, r_out in zip(S.records(pcap), S.records(out)):
        d, o = r_in[4], r_out[4]
        if _eth_of(kind, r_in, b"", b"") is None:
            assert o == d
            continue
        tci = (45 | 5 << 13).to_bytes(2, "big")
        exp = tci + b"\x00\x00" + bytes.fromhex("99aa") + bytes.fromhex("001122334455") + b"\x81\x00" + \
            d[14:18] + d[hl:]
        assert rc == 0 and o == exp


# ------------------------------------------------------------------------- GPU
ARGSETS = [
    ["--fixcsum"],
    ["--dlt=enet"] + MACS + ["--fixcsum"],
    ["--dlt=enet"] + MACS + ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353", "--fixcsum"],
    ["--dlt=enet"] + MACS + ["--seed=11", "--ttl=+2", "--efcs"],
    # (--enet-mac-seed cannot be combined with --enet-smac/--enet-dmac: dlt_en10mb.def:62-63)
    ["--dlt=enet"] + MACS + ["--enet-vlan=del", "--tos=5", "--mtu-trunc", "--mtu=400", "--fixcsum"],
    ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1", "--fixcsum"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--seed=5"],
    ["--dlt=pppserial", "--fixcsum"],
    # --fuzz-seed behind the decoder: a fuzzed record goes back to `again:`, is decoded by the
    # input decoder and encoded a second time (tcpedit.c:89,250-258); a 40-byte user header
    # needs 2 x 40 bytes of slot headroom behind DLT_RAW
    ["--dlt=enet"] + MACS + ["--fuzz-seed=7", "--fuzz-factor=2", "--fixcsum"],
    ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1", "--fuzz-seed=5",
     "--fuzz-factor=3"],
    ["--dlt=user", "--user-dlink=" + ",".join("%02x" % (b + 0x40) for b in range(38)) + ",08,00", "--user-dlt=1",
     "--fuzz-seed=11", "--fuzz-factor=1", "--fixcsum"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--fuzz-seed=9", "--fuzz-factor=2"],
    ["--fuzz-seed=3", "--fuzz-factor=1"],
    # round 5, the reference's failing encodes written half-moved (soft errors): the hdlc
    # encoder without its fields (hdlc.c:240-288), en10mb without addresses (en10mb.c:567-619),
    # and a VLAN push behind another decoder (the tag at byte 0, en10mb.c:696-715)
    ["--dlt=hdlc"],
    ["--dlt=hdlc", "--hdlc-address=15", "--seed=2"],
    ["--dlt=enet", "--fixcsum"],
    ["--dlt=enet", "--enet-smac=00:11:22:33:44:55", "--seed=6"],
    ["--dlt=enet", "--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"] +
    MACS,
    ["--dlt=enet", "--enet-vlan=add", "--enet-vlan-tag=7", "--fuzz-seed=4", "--fuzz-factor=2"] + MACS,
]


def _gpu_vs_oracle(pcap, args, dlt, cache=None):
    rc_o, exp = O.rewrite(pcap, args, cache)
    te = TA.TcpEdit(args, dlt=dlt)
    try:
        rc, out = te.rewrite(pcap, cache)
        assert (rc, out) == (rc_o, exp), args
    finally:
        te.close()
    # a fresh context: --fuzz-seed's RNG state carries from one call to the next (fuzzing.c:8-20)
    te = TA.TcpEdit(args, dlt=dlt)
    try:
        rc, out = te.rewrite_pipelined(pcap, cache, chunk_bytes=1 << 16)
        assert (rc, out) == (rc_o, exp), args
    finally:
        te.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("k", range(len(ARGSETS)))
def test_gpu_matches_oracle(built, kind, k):
    args = ARGSETS[k]
    pcap = S.reframe(_base(3000, seed=k + 1), kind, odd_every=11)
    _gpu_vs_oracle(pcap, args, DLT_OF[kind])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sll", "sll2"])
@pytest.mark.parametrize("dmac", [False, True])
def test_gpu_dst_modified_carries_across_s2c_records(built, kind, dmac):
    """behind a Linux cooked decoder, a C2S record without --enet-dmac sets the
    en10mb encoder's dst_modified and an S2C record keeps the last C2S record's value;
    the multicast MAC update of every record reads it.  Multicast destinations and
    all-zero cooked headers (dst_modified false) make the carried value visible."""
    base = S.records(_base(4000, seed=21))
    recs = []
    for i, (ts, tu, cl, ln, d) in enumerate(base):
        d = bytearray(d)
        if i % 3 == 0 and d[12:14] == b"\x08\x00":
            d[30:34] = bytes([224 + i % 16, 1, 2, 3])  # a multicast IPv4 destination
        recs.append((ts, tu, cl, ln, bytes(d)))
    pcap = bytearray(S.reframe(S.build_pcap(recs), kind))
    # zero the first 6 bytes of every 5th record's cooked header (dst_modified false there)
    off, i = 24, 0
    while off + 16 <= len(pcap):
        cl = struct.unpack_from("<I", pcap, off + 8)[0]
        if i % 5 == 0:
            if kind == "sll":
                pcap[off + 16:off + 18] = b"\x00\x00"
                pcap[off + 20:off + 22] = b"\x00\x00"  # halen 0 (address bytes stay)
            else:
                pcap[off + 16:off + 22] = bytes(6)     # ethertype + reserved + ifindex hi: zero
        off += 16 + cl
        i += 1
    pcap = bytes(pcap)
    cache = S.tcpprep_cache(len(base), seed=5, nosend_every=9)
    args = ["--dlt=enet", "--fixcsum"] + (["--enet-dmac=00:66:77:88:99:aa,01:00:5e:00:00:09"] if dmac else [])
    _gpu_vs_oracle(pcap, args, DLT_OF[kind], cache)
    # the carry crosses batches: two halves through one context equal the whole
    rc_o, exp = O.rewrite(pcap, args, cache)
    te = TA.TcpEdit(args, dlt=DLT_OF[kind])
    try:
        rc, out = te.rewrite_pipelined(pcap, cache, chunk_bytes=1 << 14)
        assert (rc, out) == (rc_o, exp)
    finally:
        te.close()


@pytest.mark.gpu
def test_gpu_per_packet_api_on_cooked_input(built):
    """tcpedit_packet with a DLT_LINUX_SLL context, record by record, equals the batch"""
    pcap = S.reframe(_base(300, seed=9), "sll", odd_every=13)
    args = ["--dlt=enet", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args, dlt=113)
    try:
        got = []
        for ts, tu, cl, ln, d in S.records(pcap):
            buf = bytearray(d) + bytearray(262166)
            rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf, 1)
            assert rc != -1, te.geterr()
            got.append((h["ts_sec"], h["ts_usec"], h["caplen"], h["len"], bytes(buf[:h["caplen"]])))
        assert got == S.records(exp)
    finally:
        te.close()
