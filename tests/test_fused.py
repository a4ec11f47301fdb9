"""The window mode of the wave lane (tcpedit_batch_run_fused): the record discovery fused
into the edit -- each wave stages a byte window of the capture, finds its records
(te_window.hpp, the same speculation te_index.hip makes), cuts them into tiles and edits
them where they lie; te_win_check then checks the chain across windows.  Every case must
write the oracle's bytes; a batch the window mode does not carry, or one where the
speculation misses the chain, runs the exact path (tcpedit_batch_run) instead."""
import ctypes
import struct

import pytest

import fl_cases as F
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu


def _run(pcap, args, cache=None, fused=True):
    """fused: True -> the window mode must carry the batch, False -> it must not, None -> either"""
    rc_o, exp = O.rewrite(pcap, args, cache)
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap, cache)
        rc = b.run_fused()
        out, r, fb = b.output(), b.result(), b.fused_fallbacks
        st = b.status()
        t = b.time_fused(2)
        b.close()
    finally:
        te.close()
    assert rc == rc_o
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"
    if fused is True:
        assert fb == 0 and t is not None and t > 0
        assert r.packets == len(S.records(pcap)) and not st.any()
    elif fused is False:
        assert t is None or fb == 1
    return fb, r


@pytest.mark.parametrize("name,gen,args", [
    ("c2", lambda: S.pcap_fixed(100_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
    ("c2-plain", lambda: S.pcap_fixed(50_000, 64, seed=2), ["--fixcsum"]),
    ("imix", lambda: S.pcap_imix(60_000, seed=3), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353",
                                                   "--fixcsum"]),
    ("ipmap", lambda: S.pcap_imix(30_000, seed=4), ["--srcipmap=10.0.0.0/8:172.16.0.0/12", "--fixcsum"]),
    ("c5", lambda: S.pcap_mixed_v4v6(20_000, 1514, seed=5), ["--fixcsum"]),
    ("macs", lambda: S.pcap_imix(30_000, seed=6), ["--enet-smac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee",
                                                   "--enet-dmac=00:66:77:88:99:aa,00:12:34:56:78:9a",
                                                   "--ttl=+3", "--tos=7", "--fixcsum"]),
    # the incremental-checksum instances (no --fixcsum)
    ("seed-incr", lambda: S.pcap_fixed(40_000, 64, seed=7), ["--seed=42"]),
    ("hdr-incr", lambda: S.pcap_imix(30_000, seed=8), ["--ttl=+1", "--tos=7"]),
    ("all-incr", lambda: S.pcap_imix(30_000, seed=9), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353",
                                                       "--enet-dmac=00:66:77:88:99:aa,00:12:34:56:78:9a",
                                                       "--ttl=9"]),
    ("v6", lambda: S.pcap_fixed(20_000, 200, ipv6=True, proto=6, seed=10), ["--seed=5", "--fixcsum"]),
], ids=lambda x: x if isinstance(x, str) else "")
def test_fused_matches_the_oracle(built, name, gen, args):
    _run(gen(), args)


def test_fused_mixed_records(built):
    """ARP, IPv6 extension headers, fragments, non-IP: records the wave lane defers send
    the batch to the exact path; the bytes are the oracle's either way"""
    _run(F.build(F.mixed(8000, seed=7)), ["--seed=7", "--fixcsum"], fused=None)


def test_fused_records_larger_than_a_window(built):
    """records of 9000 and 40000 bytes between small ones: a window's last record reaching
    past its staged bytes is loaded after it (<= 2 KiB) or left to the exact path"""
    base = S.records(S.pcap_fixed(3000, 90, seed=9))
    mid = S.records(S.pcap_fixed(4, 1800, seed=8))
    big = S.records(S.pcap_fixed(3, 9000, seed=10)) + S.records(S.pcap_fixed(2, 40000, seed=11))
    recs = []
    for i, r in enumerate(base):
        recs.append(r)
        if i % 53 == 0:
            recs.append(mid[(i // 53) % len(mid)])
    _run(S.build_pcap(recs), ["--seed=3", "--fixcsum"], fused=None)
    for i, r in enumerate(big):
        recs.insert(500 + 700 * i, r)
    _run(S.build_pcap(recs), ["--seed=3", "--fixcsum"], fused=None)


def test_fused_chain_ends(built):
    """a truncated last record, an oversize record (libpcap stops), a len > 262144 record and
    records with caplen 0, len 0 or both (safe_pcap_next's exit, src/common/utils.c:136-156:
    the output ends before them, rc -1), and a len < caplen record (the reader trims its
    caplen to len, utils.c:159-162): all taken by the exact path"""
    recs = S.records(S.pcap_fixed(20_000, 80, seed=12))
    pcap = S.build_pcap(recs)
    _run(pcap[:-30], ["--fixcsum"], fused=None)
    ts, tu, cl, ln, d = recs[12_345]
    over = S.build_pcap(recs[:12_345]) + struct.pack("<IIII", ts, tu, 300_000, 300_000) + d + \
        S.build_pcap(recs[12_346:])[24:]
    _run(over, ["--fixcsum"], fused=False)
    err = S.build_pcap(recs[:9_999] + [(ts, tu, cl, 400_000, d)] + recs[10_000:])
    _run(err, ["--fixcsum"], fused=False)
    for zc, zl in ((0, 0), (0, 80), (cl, 0)):
        zero = S.build_pcap(recs[:5000] + [(ts, tu, zc, zl, d[:zc])] + recs[5000:])
        _run(zero, ["--fixcsum"], fused=False)
    trim = S.build_pcap(recs[:7000] + [(ts, tu, cl, cl - 9, d)] + recs[7000:])
    _run(trim, ["--fixcsum"], fused=False)


def test_fused_record_like_payloads(built):
    """payloads full of valid-looking record headers: a guess may land inside a packet; the
    chain check either repairs it or sends the batch to the exact path"""
    fake = b"".join(struct.pack("<IIII", 1, 2, 12, 12) + bytes(range(12)) for _ in range(50))
    recs = []
    for ts, tu, cl, ln, d in S.records(S.pcap_fixed(4_000, 1_442, seed=13)):
        d = bytearray(d)
        d[42:42 + len(fake)] = fake
        recs.append((ts, tu, cl, ln, bytes(d)))
    _run(S.build_pcap(recs), ["--seed=3", "--fixcsum"], fused=None)


@pytest.mark.parametrize("args,cache", [
    (["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"], False),
    (["--efcs", "--ttl=3"], False),
    (["--fixlen=pad", "--fixcsum"], False),
    (["--endpoints=10.10.0.1:10.10.0.2", "--fixcsum"], True),
], ids=["vlan-add", "efcs", "fixlen", "cache"])
def test_fused_not_carried(built, args, cache):
    """size-changing configs, generic-lane configs and a tcpprep cache run the exact path"""
    pcap = S.pcap_imix(10_000, seed=14)
    c = S.tcpprep_cache(10_000, seed=14, nosend_every=7) if cache else None
    _run(pcap, args, c, fused=False)


def test_fused_not_carried_inputs(built):
    """big-endian and nanosecond captures run the exact path (the window mode reads native
    microsecond headers only)"""
    recs = S.records(S.pcap_imix(8_000, seed=17))
    for magic in (0xA1B23C4D, 0xD4C3B2A1):
        sw = magic == 0xD4C3B2A1
        e = ">" if sw else "<"
        hdr = struct.pack(e + "IHHiIII", 0xA1B2C3D4 if sw else magic, 2, 4, 0, 0, 65535, 1)
        body = b"".join(struct.pack(e + "IIII", ts, tu * (1000 if magic == 0xA1B23C4D else 1), cl, ln) + d
                        for ts, tu, cl, ln, d in recs)
        _run(hdr + body, ["--seed=5", "--fixcsum"], fused=False)


def test_fused_small_and_empty(built):
    """one record, a few records (fewer windows than waves), the file header alone"""
    recs = S.records(S.pcap_fixed(50, 200, seed=15))
    for n in (1, 3, 50):
        _run(S.build_pcap(recs[:n]), ["--seed=9", "--fixcsum"])
    _run(S.build_pcap([]), ["--fixcsum"], fused=None)


def test_fused_runs_repeat(built):
    """the same batch run twice (window workspace reused) and after a config change"""
    pcap = S.pcap_imix(20_000, seed=16)
    args = ["--seed=11", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap)
        for _ in range(2):
            assert b.run_fused() == rc_o and b.output() == exp
        assert b.fused_fallbacks == 0
        b.close()
    finally:
        te.close()


def _udp_frame(size, payload_at=None, payload=b""):
    """an Ethernet II / IPv4 / UDP frame of `size` bytes (checksums left to --fixcsum), with
    `payload` written at frame offset payload_at and 0xEE filler elsewhere in the UDP payload
    (no zero bytes: nothing there looks like a record header to the discovery)"""
    f = bytearray(b"\xee" * size)
    f[0:14] = bytes.fromhex("001122334455" "00667788 99aa".replace(" ", "")) + b"\x08\x00"
    f[14:34] = struct.pack(">BBHHHBBH4s4s", 0x45, 0, size - 14, 1, 0x4000, 64, 17, 0, bytes([10, 1, 2, 3]),
                           bytes([172, 16, 0, 9]))
    f[34:42] = struct.pack(">HHHH", 4000, 53, size - 34, 0)
    if payload_at is not None:
        f[payload_at:payload_at + len(payload)] = payload
    return bytes(f)


def _fake_chain():
    """pcap records as payload bytes: five 64-byte UDP records, an ARP record (a shape the
    wave lane leaves to the exact path) and the header of a 6,000-byte record (past the
    window's staged tail: also left to the exact path)"""
    parts = []
    for i in range(5):
        parts.append(struct.pack("<IIII", 1700000000, 1000 + i, 64, 64) + _udp_frame(64))
    arp = bytes.fromhex("ffffffffffff" "00667788 99aa".replace(" ", "")) + b"\x08\x06" + b"\x00\x01" * 23
    parts.append(struct.pack("<IIII", 1700000000, 2000, len(arp), len(arp)) + arp)
    parts.append(struct.pack("<IIII", 1700000000, 3000, 6000, 6000))
    return b"".join(parts)


def test_window_pipeline_false_records_before_the_chain_entry(built):
    """in the window-mode pipeline the windows before a chunk's chain entry (kE)
    hold the tail of the previous chunk's last record; what the discovery finds there is not
    a record, the edit's writes there are overwritten by the head copy, and a record it
    leaves to the exact path (WIN_F_EDIT) must not send the capture to the fallback.  Here the
    record straddling the first chunk cut is a 5,050-byte UDP frame (the lean window tile
    holds it) whose payload past the cut carries a fake record chain with a deferred ARP
    record and an over-long record: the output is the oracle's and no call falls back."""
    args = ["--seed=42", "--fixcsum"]
    n_total = (3 << 20) + 4096
    buf = bytearray(n_total)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    # te_api.c win_plan: the first chunk cut at a 256-byte boundary of the caller's buffer
    # 1 MiB past the first record (1 MiB chunks)
    cut1 = ((addr + 24 + (1 << 20)) & ~255) - addr
    # the jumbo: 16 + J + 16 within the 5,120-byte lean window tile; its bytes past the cut,
    # 16 + J - 100 = 4,966, put the next chunk's chain entry in its window 1 (kE = 1).  (Its
    # chunk-0 window offset is 1,660-1,916 for any buffer address: the window's staging plus
    # its tail load hold the whole record.)
    J = 5050
    jstart = cut1 - 100
    recs, off, i = [], 24, 0
    while off < jstart:
        gap = jstart - off
        size = 64 if gap >= 80 + 76 or gap == 80 else gap - 16  # (the last filler 60..139 bytes)
        recs.append((1600000000, i, size, size, _udp_frame(size)))
        off += 16 + size
        i += 1
    assert off == jstart
    fake = _fake_chain()
    # chunk-1 offset 200 is jumbo data offset 200 + 84
    recs.append((1600000001, 0, J, J, _udp_frame(J, 284, fake)))
    off += 16 + J
    while off + 80 <= n_total:
        recs.append((1600000002, i, 64, 64, _udp_frame(64)))
        off += 80
        i += 1
    pcap = S.build_pcap(recs)
    assert len(pcap) <= n_total
    buf[:len(pcap)] = pcap  # (in place: the address the cut was computed for)
    src = memoryview(buf)[:len(pcap)]
    rc_o, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args)
    try:
        rc, out = te.rewrite_pipelined(src, chunk_bytes=1 << 20)
        assert rc == rc_o == 0
        assert out == exp
        assert te.pipeline_fallbacks == 0
        src.release()
    finally:
        te.close()
