"""The window mode of the wave lane (tcpedit_batch_run_fused): the record discovery fused
into the edit -- each wave stages a byte window of the capture, finds its records
(te_window.hpp, the same speculation te_index.hip makes), cuts them into tiles and edits
them where they lie; te_win_check then checks the chain across windows.  Every case must
write the oracle's bytes; a batch the window mode does not carry, or one where the
speculation misses the chain, runs the exact path (tcpedit_batch_run) instead."""
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
