"""The Juniper Ethernet, 802.11 and radiotap decoders: DLT_JUNIPER_ETHER
(src/tcpedit/plugins/dlt_jnpr_ether/jnpr_ether.c), DLT_IEEE802_11 (dlt_ieee80211/ieee80211.c,
ieee80211_hdr.c) and DLT_IEEE802_11_RADIO (dlt_radiotap/radiotap.c), as decoders into the
en10mb encoder (--dlt=enet) and into their own plugins (which refuse to encode).

Parity is unpinned: the reference ships no capture of these link types.  The oracle's
restatement (oracle/tcpedit_oracle.c jnpr_*, i80211_*, the radiotap proto) is checked here
against outputs built independently from the synthetic framings (CPU), and the GPU against
the oracle, bit-exact.  Reference behaviours kept:
  * radiotap: dlt_radiotap_get_80211 copies the 802.11 frame into its MAXPACKET extra
    buffer only when the frame is at least that long, so the 802.11 proto reads zeros and
    every record is a soft error, written as read (radiotap.c:344-364);
  * 802.11: frame control read with ntohs; the source/destination by the DS bits; the
    SNAP type as the proto; management, protected and non-SNAP frames are soft errors;
  * Juniper: the inner Ethernet frame's en10mb decode supplies addresses, proto and the
    VLAN fields (by the extra pointer), so --enet-vlan=del writes the inner type and a
    tagged inner frame without --enet-vlan gets its TCI written at offset 14 of the new
    frame; a frame whose extensions are not Ethernet is a TCPEDIT_WARN (jnpr_ether.c:269-272)
    that is encoded with the state the last whole inner decode left in the context (its
    addresses and proto, dlt_utils.c:249-271, and by the extra pointer the sub-decoder's
    VLAN fields) -- zeros before the first, whose sub-decoder extra then becomes the
    encoder's (a fresh dst_modified).  The device carries it with a mark + max scan over
    the records (te_jnpr_mark), across launches, pipeline chunks and shards."""
import struct

import pytest

import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

KINDS = list(S.LINKTYPES_MORE)
DLT_OF = {"jnpr": 178, "80211": 105, "radiotap": 127}
MACS = ["--enet-smac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee", "--enet-dmac=00:66:77:88:99:aa,00:12:34:56:78:9a"]
DMAC, SMAC = bytes.fromhex("00667788" "99aa"), bytes.fromhex("001122334455")


def _base(n=600, seed=3):
    return S.pcap_imix(n, seed=seed)


def _w80211_ok(d):
    fc = d[0] << 8 | d[1]
    if (fc & 0x0F00) != 0x0800 or (fc & 0x40):
        return None
    h = (2 if fc & 0x8000 else 0) + (30 if fc & 3 == 3 else 24)
    if d[h:h + 2] != b"\xaa\xaa":
        return None
    return h + 8, d[h + 6:h + 8]


@pytest.mark.parametrize("kind", KINDS)
def test_oracle_own_encoder_writes_the_capture_unedited(built, kind):
    """no --dlt: the decoder's own plugin refuses to encode -- every record a soft error,
    written as read; with --skip-soft-errors nothing is written"""
    pcap = S.reframe(_base(), kind, odd_every=7)
    rc, out = O.rewrite(pcap, ["--fixcsum", "--seed=7"])
    assert rc == 0 and S.records(out) == S.records(pcap)
    assert int.from_bytes(out[20:24], "little") == DLT_OF[kind]
    rc, out = O.rewrite(pcap, ["--fixcsum", "--skip-soft-errors"])
    assert rc == 0 and S.records(out) == []


def test_oracle_radiotap_is_always_a_soft_error(built):
    pcap = S.reframe(_base(), "radiotap")
    rc, out = O.rewrite(pcap, ["--dlt=enet"] + MACS + ["--fixcsum"])
    assert rc == 0 and S.records(out) == S.records(pcap)
    assert int.from_bytes(out[20:24], "little") == 1


def test_oracle_80211_into_ethernet_matches_the_layout(built):
    """data frames become {the given MACs, the SNAP type, the L3 bytes}; management,
    protected and non-SNAP frames are written as read"""
    pcap = S.reframe(_base(), "80211", odd_every=7)
    rc, out = O.rewrite(pcap, ["--dlt=enet"] + MACS)
    assert rc == 0
    exp = []
    for ts, tu, cl, ln, d in S.records(pcap):
        ok = _w80211_ok(d)
        if ok is None:
            exp.append((ts, tu, cl, ln, d))
            continue
        hl, et = ok
        nd = DMAC + SMAC + et + d[hl:]
        exp.append((ts, tu, cl + len(nd) - len(d), ln + len(nd) - len(d), nd))
    assert S.records(out) == exp


def test_oracle_80211_addresses_by_ds_bits(built):
    """without --enet-smac/--enet-dmac the 802.11 source and destination are written:
    addr2/addr3 (no DS bit, ToDS), addr3/addr1 (FromDS), addr4/addr3 (both)"""
    pcap = S.reframe(_base(80), "80211")
    rc, out = O.rewrite(pcap, ["--dlt=enet"])
    assert rc == 0
    for r_in, r_out in zip(S.records(pcap), S.records(out)):
        d, o = r_in[4], r_out[4]
        ds = d[1] & 3
        src = {0: d[10:16], 1: d[10:16], 2: d[16:22], 3: d[24:30]}[ds]
        dst = {0: d[16:22], 1: d[16:22], 2: d[4:10], 3: d[16:22]}[ds]
        assert o[:6] == dst and o[6:12] == src


def test_oracle_jnpr_into_ethernet_strips_header_and_tag(built):
    """--enet-vlan=del: the Juniper header and the inner Ethernet header (with its 802.1Q
    tag) become {the given MACs, the inner L3 type}; bad-magic records stay as read"""
    base = S.records(_base())
    pcap = S.reframe(S.build_pcap(base), "jnpr", odd_every=7)
    rc, out = O.rewrite(pcap, ["--dlt=enet", "--enet-vlan=del"] + MACS)
    assert rc == 0
    exp = []
    for k, ((ts, tu, cl, ln, d), (_, _, _, _, e)) in enumerate(zip(S.records(pcap), base)):
        if d[:3] != b"\x4d\x47\x43":
            exp.append((ts, tu, cl, ln, d))
            continue
        nd = DMAC + SMAC + e[12:]
        exp.append((ts, tu, cl + len(nd) - len(d), ln + len(nd) - len(d), nd))
    assert S.records(out) == exp


def test_fuzz_with_the_dst_modified_carry_is_served(built):
    # (--fuzz-seed with the en10mb encoder's dst_modified carry, SURVEY Q18: no --enet-dmac;
    # refused through round 4, served by the carry's mark run of the edit since round 5)
    for dlt, args in [(105, ["--fuzz-seed=3", "--dlt=enet"]), (178, ["--fuzz-seed=3", "--dlt=enet"])]:
        TA.TcpEdit(args, dlt=dlt).close()


# ------------------------------------------- Q18 under --fuzz-seed: the second encode writes
def _cache_of(dirs):
    """a tcpprep v04 cache (cache.h:63-72) from per-record directions (1 C2S, 2 S2C)"""
    body = bytearray((len(dirs) + 3) // 4)
    for i, d in enumerate(dirs):
        body[i // 4] |= (0b11 if d == 1 else 0b10) << (2 * (i % 4))
    return b"tcpprep\0" + b"04\0\0" + struct.pack(">QHH", len(dirs), 4, 0) + bytes(body)


def q18_fuzz_capture(n=1500, seed=5):
    """802.11 data frames (ToDS = FromDS = 0: destination = addr3, tcpedit's
    ieee80211_get_dst) around IPv4/UDP, in four kinds, with their directions:
      A  C2S; addr3 = the frame's first 6 bytes (FC, duration, addr1[0:2]), so the first
         encode writes dst_modified = 0; the IP checksum is 0xAAAA, so the second decode
         (tcpedit.c:89: the re-encoded Ethernet frame read as 802.11 -- its destination
         08:00:.. a data frame control word, SNAP at the IP checksum) succeeds and the second
         encode writes dst_modified = 1 (en10mb.c:614)
      B  C2S as A but an ordinary checksum: the second decode fails, the carry stays 0
      C  S2C, second decode as A, the UDP payload's bytes 6..9 a multicast address that the
         second pass reads as the IPv4 destination: its multicast MAC update (en10mb.c:
         868-873) shows the carried value
      D  C2S, addr3 not the first 6 bytes (dst_modified = 1), second decode fails
    Every record reaches the fuzz step, so every one goes through the second pass; a high
    --fuzz-factor fuzzes few of them."""
    import numpy as np
    rng = np.random.default_rng(seed)
    recs, dirs, kinds = [], [], []
    for i in range(n):
        k = "ABCD"[int(rng.integers(0, 4))] if i else "A"
        plen = int(rng.integers(16, 120))
        pay = bytearray(rng.integers(0, 256, plen, dtype=np.uint8).tobytes())
        pay[6:10] = bytes([224 + i % 16, 1, 2, 3])
        ulen = 8 + plen
        udp = struct.pack(">HHHH", int(rng.integers(1024, 65535)), 53, ulen, 0x12FD)
        dst_ip = bytes([8, 0, 0x45, int(rng.integers(0, 256))])
        csum = b"\xaa\xaa" if k in "AC" else b"\x12\x34"
        ip = (bytes([0x45, 0]) + struct.pack(">HH", 20 + ulen, i & 0xFFFF) + b"\x40\x00\x40\x11" + csum +
              bytes([10, 1, int(rng.integers(0, 256)), int(rng.integers(0, 256))]) + dst_ip)
        dur = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()
        a1 = rng.integers(0, 256, 6, dtype=np.uint8).tobytes()
        a2 = bytes([2]) + rng.integers(0, 256, 5, dtype=np.uint8).tobytes()
        a3 = b"\x08\x00" + dur + a1[:2]
        if k == "D":
            a3 = b"\x08\x00" + bytes([dur[0] ^ 0x5A]) + a3[3:]
        frame = b"\x08\x00" + dur + a1 + a2 + a3 + b"\x10\x00" + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + ip + udp + bytes(pay)
        recs.append((1600000000 + i // 1000, i % 1000 * 1000, len(frame), len(frame), frame))
        dirs.append(2 if k == "C" else 1)
        kinds.append(k)
    return S.build_pcap(recs, 105), _cache_of(dirs), kinds


Q18_FZ_ARGS = ["--dlt=enet", "--fuzz-seed=9", "--fuzz-factor=64"]


def test_oracle_second_encode_writes_the_carry(built):
    """the restatement keeps the second encode's dst_modified write: an S2C record after an
    A (first encode 0, second 1) skips the multicast MAC update, one after a B (0, no second
    encode) takes it -- so a carry found from the first encodes alone would be wrong"""
    pcap, cache, kinds = q18_fuzz_capture()
    # (a factor no draw divides: no record is fuzzed, every one goes through the second pass)
    rc, out = O.rewrite(pcap, Q18_FZ_ARGS[:2] + ["--fuzz-factor=1000000000"], cache)
    assert rc == 0
    got = S.records(out)
    assert len(got) == len(kinds)
    last, seen = None, {"A": 0, "B": 0}
    for k, (_, _, _, _, d) in zip(kinds, got):
        if k in "ABD":
            last = k
            continue
        if last in ("A", "B"):
            upd = d[:3] == b"\x01\x00\x5e"
            assert upd == (last == "B"), (last, d[:6].hex())
            seen[last] += 1
    assert seen["A"] > 20 and seen["B"] > 20


# ------------------------------------------------------------------------- GPU
ARGSETS = [
    ["--fixcsum"],
    ["--dlt=enet"] + MACS + ["--fixcsum"],
    ["--dlt=enet"] + MACS + ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353", "--fixcsum"],
    ["--dlt=enet"] + MACS + ["--seed=11", "--ttl=+2", "--efcs"],
    ["--dlt=enet", "--enet-vlan=del", "--tos=5", "--mtu-trunc", "--mtu=400", "--fixcsum"] + MACS,
    ["--dlt=enet", "--seed=3", "--fixcsum"],  # the decoded addresses (802.11, Juniper's inner frame)
    ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1", "--fixcsum"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--seed=5"],
    # --fuzz-seed behind the decoder: a fuzzed record is decoded and encoded twice
    # (tcpedit.c:89,250-258)
    ["--dlt=enet", "--fuzz-seed=3", "--fuzz-factor=2", "--fixcsum"] + MACS,
    ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1", "--fuzz-seed=5",
     "--fuzz-factor=1"],
    ["--fuzz-seed=4", "--fuzz-factor=1"],
    ["--dlt=enet", "--enet-vlan=add", "--enet-vlan-tag=9", "--fixcsum"] + MACS,
    ["--dlt=hdlc", "--seed=8"],
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
    pcap = S.reframe(_base(3000, seed=k + 1), kind, odd_every=11)
    _gpu_vs_oracle(pcap, ARGSETS[k], DLT_OF[kind])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["jnpr", "80211"])
def test_gpu_dst_modified_carries_across_s2c_records(built, kind):
    """SURVEY Q18 behind these decoders: a C2S record without --enet-dmac sets the en10mb
    encoder's dst_modified (the frame's first 6 bytes against the decoded destination), an
    S2C record keeps the last C2S record's value, the multicast MAC update reads it"""
    base = S.records(_base(4000, seed=21))
    recs = []
    for i, (ts, tu, cl, ln, d) in enumerate(base):
        d = bytearray(d)
        if i % 3 == 0 and d[12:14] == b"\x08\x00":
            d[30:34] = bytes([224 + i % 16, 1, 2, 3])
        recs.append((ts, tu, cl, ln, bytes(d)))
    pcap = S.reframe(S.build_pcap(recs), kind)
    cache = S.tcpprep_cache(len(base), seed=5, nosend_every=9)
    args = ["--dlt=enet", "--fixcsum"]
    _gpu_vs_oracle(pcap, args, DLT_OF[kind], cache)


@pytest.mark.gpu
def test_gpu_second_encode_writes_the_carry(built):
    """SURVEY Q18 under --fuzz-seed: the carry's mark run of the edit finds each record's
    last dst_modified write, the second encode's included -- batch and 16 KiB pipeline
    chunks equal the oracle"""
    pcap, cache, _ = q18_fuzz_capture()
    _gpu_vs_oracle(pcap, Q18_FZ_ARGS[:2] + ["--fuzz-factor=1000000000"], 105, cache)
    _gpu_vs_oracle(pcap, Q18_FZ_ARGS, 105, cache)
    rc_o, exp = O.rewrite(pcap, Q18_FZ_ARGS, cache)
    te = TA.TcpEdit(Q18_FZ_ARGS, dlt=105)
    try:
        rc, out = te.rewrite_pipelined(pcap, cache, chunk_bytes=1 << 14)
        assert (rc, out) == (rc_o, exp)
    finally:
        te.close()


@pytest.mark.gpu
def test_gpu_second_encode_carry_per_packet(built):
    """the same through tcpedit_packet, record by record with each record's direction: the
    carry and the RNG state cross the calls in the context (launch per call)"""
    pcap, cache, kinds = q18_fuzz_capture(400, seed=6)
    args = Q18_FZ_ARGS[:2] + ["--fuzz-factor=1000000000"]
    rc_o, exp = O.rewrite(pcap, args, cache)
    te = TA.TcpEdit(args, dlt=105)
    try:
        got = []
        for k, (ts, tu, cl, ln, d) in zip(kinds, S.records(pcap)):
            buf = bytearray(d) + bytearray(262166)
            rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf, 2 if k == "C" else 1)
            assert rc != -1, te.geterr()
            got.append((h["ts_sec"], h["ts_usec"], h["caplen"], h["len"], bytes(buf[:h["caplen"]])))
        assert got == S.records(exp)
    finally:
        te.close()


def _jnpr_warn(n=600, seed=4, every=7, lead=3, cut=None):
    """a Juniper capture whose records lead, lead + 1, ... (the first `lead` records, then
    every `every`-th) carry encapsulation 15 (not Ethernet: TCPEDIT_WARN); every 4th inner
    frame is 802.1Q-tagged (S.reframe), so the carried VLAN fields change along the way"""
    recs = S.records(S.reframe(_base(n, seed=seed), "jnpr"))
    warn = set(range(lead)) | {i for i in range(len(recs)) if i % every == 2}
    for i in sorted(warn):
        ts, tu, cl, ln, d = recs[i]
        d = bytearray(d)
        k = d.find(b"\x06\x01\x0e")
        d[k + 2] = 0x0f
        # the warning frame's l2len is the Juniper header alone, so an encoder takes the inner
        # Ethernet header for the L3 bytes; a first byte of 0x45 keeps them an IPv4 header
        # (version 4 is what --fixcsum demands, edit_packet.c:73-79: else the run stops there)
        hl = 6 + (d[4] << 8 | d[5])
        d[hl] = 0x45
        recs[i] = (ts, tu, cl, ln, bytes(d))
    return S.build_pcap(recs, 178), warn


JMAGIC_DMAC = "4d:47:43:80:00:00"  # the Juniper magic + L2-present flag + no extensions


@pytest.mark.gpu
@pytest.mark.parametrize("q18", [False, True])
def test_gpu_second_decode_is_a_juniper_warning_frame(built, q18):
    """--fuzz-seed behind the Juniper decoder into --dlt=enet, where the re-encoded frame
    starts with the Juniper magic (its destination 4d:47:43:80:00:00: a header of 6 bytes and
    no extensions), so every record's second decode (tcpedit.c:89,250-258) is a TCPEDIT_WARN
    frame, encoded with the state its own first pass left (its whole inner decode, else the
    carried one).  q18: the destination is the inner frame's own (no --enet-dmac), so the
    dst_modified carry's mark run goes through those second encodes too.  Refused through
    round 4; parity is unpinned (no reference capture), the oracle restates the sequence."""
    pcap, _ = _jnpr_warn(700, seed=12)
    if q18:
        recs = []
        for ts, tu, cl, ln, d in S.records(pcap):
            d = bytearray(d)
            hl = 6 + (d[4] << 8 | d[5])
            if hl + 6 <= len(d):
                d[hl:hl + 6] = bytes.fromhex(JMAGIC_DMAC.replace(":", ""))
            recs.append((ts, tu, cl, ln, bytes(d)))
        pcap = S.build_pcap(recs, 178)
        args = ["--dlt=enet", "--enet-smac=00:11:22:33:44:55", "--fuzz-seed=3", "--fuzz-factor=4"]
        cache = _cache_of([1 + (i % 3 == 1) for i in range(len(recs))])
    else:
        args = ["--dlt=enet", "--enet-dmac=" + JMAGIC_DMAC, "--enet-smac=00:11:22:33:44:55", "--fuzz-seed=5",
                "--fuzz-factor=3"]
        cache = None
    rc_o, exp = O.rewrite(pcap, args, cache)
    assert rc_o == 0
    _gpu_vs_oracle(pcap, args, 178, cache)


def test_oracle_jnpr_warning_frames_encode_with_the_carried_state(built):
    """--dlt=enet with both MACs: a warning frame gets a new Ethernet header in place of its
    Juniper header (only that header is its l2len), whose type is the carried proto -- the
    last whole decode's inner ethertype, zero before the first"""
    pcap, warn = _jnpr_warn(200)
    args = ["--dlt=enet"] + MACS
    rc, out = O.rewrite(pcap, args)
    assert rc == 0
    prev = b"\x00\x00"
    for i, (r_in, r_out) in enumerate(zip(S.records(pcap), S.records(out))):
        d, o = r_in[4], r_out[4]
        hl = 6 + (d[4] << 8 | d[5])
        inner = d[hl:]
        if i in warn:
            # (a carried tagged decode also writes its TCI at offset 14)
            assert o[12:14] == prev and (prev == b"\x81\x00" or o[14:] == inner), i
            continue
        prev = inner[12:14]  # (en10mb.c:431: the outer type, 0x8100 for a tagged frame)


def test_oracle_jnpr_into_hdlc_fails_after_the_first_whole_decode(built):
    """--dlt=hdlc: before the first whole inner decode a warning frame becomes {address,
    control, proto 0} + the frame after its Juniper header; from that decode on the context's
    decoded extra is the en10mb sub-decoder's (dlt_utils.c:262-263), smaller than the
    hdlc_extra_t dlt_hdlc_encode demands (hdlc.c:237-238): every record is a soft error,
    written as read (tcpedit.c:104-108)"""
    pcap, warn = _jnpr_warn(200, lead=3)
    rc, out = O.rewrite(pcap, ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3"])
    assert rc == 0
    for i, (r_in, r_out) in enumerate(zip(S.records(pcap), S.records(out))):
        d, o = r_in[4], r_out[4]
        if i < 3:
            hl = 6 + (d[4] << 8 | d[5])
            assert o == bytes([15, 3, 0, 0]) + d[hl:], i
        else:
            assert r_out == r_in, i


# the option lines of the Juniper warning frames: the en10mb encoder with both MACs, with a
# VLAN pop (the carried inner type), without MACs (the carried addresses, SURVEY Q18 with a
# cache), the user and hdlc encoders, --fuzz-seed behind it
JNPR_LINES = [
    ["--dlt=enet"] + MACS + ["--fixcsum"],
    ["--dlt=enet", "--enet-vlan=del", "--seed=3"] + MACS,
    ["--dlt=enet", "--fixcsum"],
    ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1", "--ttl=9"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--seed=5"],
    ["--dlt=enet", "--fuzz-seed=3", "--fuzz-factor=2", "--fixcsum"] + MACS,
    # round 5: a VLAN push behind the Juniper decoder (the tag at the inner frame's
    # vlan_offset, en10mb.c:696-715) and the hdlc encoder without its fields
    ["--dlt=enet", "--enet-vlan=add", "--enet-vlan-tag=12", "--enet-vlan-pri=2", "--fixcsum"] + MACS,
    ["--dlt=hdlc", "--hdlc-control=3"],
]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(JNPR_LINES)))
def test_gpu_jnpr_warning_frames_match_oracle(built, k):
    """batch (one launch), pipelined (64 KiB chunks: the state crosses chunk cuts) and a
    tcpprep cache (NOSEND records decode nothing, S2C records keep Q18's value)"""
    pcap, _ = _jnpr_warn(3000, seed=k + 5)
    _gpu_vs_oracle(pcap, JNPR_LINES[k], 178)
    if "--fuzz-seed=3" not in JNPR_LINES[k]:
        cache = S.tcpprep_cache(3000, seed=k + 5, nosend_every=9)
        _gpu_vs_oracle(pcap, JNPR_LINES[k], 178, cache)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 2, 4])
def test_gpu_jnpr_warning_frames_per_packet(built, k):
    """tcpedit_packet record by record (the launch path: the server declines this config):
    the state carries from one call to the next"""
    pcap, _ = _jnpr_warn(150, seed=11)
    args = JNPR_LINES[k]
    rc_o, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args, dlt=178)
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


@pytest.mark.gpu
def test_gpu_jnpr_state_unknown_fails_loudly(built):
    """a context told its carried state is not known (a shard seeded with unknown = 1)
    fails the run at a warning frame before the shard's first whole decode"""
    pcap, _ = _jnpr_warn(200, seed=4)
    te = TA.TcpEdit(["--dlt=enet"] + MACS, dlt=178)
    try:
        te.set_jnpr_state(None, unknown=True)
        rc, out = te.rewrite(pcap)
        assert rc == -1 and "record 1" in te.geterr()
    finally:
        te.close()
