"""GPU parity for the tcpprep classification pass (tcpreplay_amd.tcpprep ->
libtcpedit_hip.so tp_classify) against the reference's own cache files and
against the CPU oracle (oracle/tcpprep_oracle.c) on adversarial and full-size
synthetic captures.  Bit-exact throughout."""
import numpy as np
import pytest

import oracle_lib
import tcpprep_cases as T
from tcpreplay_amd import synth
from tcpreplay_amd import tcpprep as TP

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(T.CASES))
def test_gpu_matches_reference_cache(name):
    assert TP.cache(T.test_pcap(), T.args(name)) == T.golden(name)


def _adversarial(seed=7, copies=6):
    """test.pcap's records (VLAN, MPLS, EoMPLS, IPv6, ARP, 802.3, padded frames) plus
    mutated copies: truncated captures (caplen 1..70), len < caplen (the reader trims caplen
    to len, src/common/utils.c:159-162), ethertypes flipped to VLAN/QinQ/IPv6/IPv4, random IP
    header bytes and v6 next-header chains."""
    rng = np.random.default_rng(seed)
    base = synth.records(T.test_pcap())
    recs = list(base)
    for _ in range(copies):
        for ts, tu, cl, ln, data in base:
            d = bytearray(data)
            k = rng.integers(0, 7)
            if k == 0 and cl:
                cl = int(rng.integers(1, min(cl, 70) + 1))
                d = d[:cl]
            elif k == 6 and cl > 1:
                recs.append((ts, tu, cl, int(rng.integers(1, cl)), bytes(d)))
                continue
            elif k == 1 and cl >= 14:
                d[12:14] = [(0x81, 0x00), (0x88, 0xa8), (0x86, 0xdd), (0x08, 0x00), (0x91, 0x00)][rng.integers(0, 5)]
            elif k == 2 and cl > 40:
                for _ in range(4):
                    d[int(rng.integers(14, min(cl, 60)))] = int(rng.integers(0, 256))
            elif k == 3 and cl > 60:
                d[12:14] = (0x86, 0xdd)
                d[14] = 0x60
                d[20] = [0, 43, 44, 60, 6, 17, 41, 59][rng.integers(0, 8)]
                d[54] = [6, 17, 0, 60][rng.integers(0, 4)]
                d[55] = int(rng.integers(0, 4))
            elif k == 4 and cl >= 12:
                d[6:12] = bytes.fromhex("001ff33ce113") if rng.integers(0, 2) else bytes.fromhex("0a0b0c0d0e0f")
            recs.append((ts, tu, len(d), max(ln, len(d)), bytes(d)))
    return synth.build_pcap(recs)


OPTION_LINES = [
    ["--cidr=96.17.211.0/24,10.0.0.0/8"],
    ["--cidr=96.17.211.0/24", "--reverse", "--nonip"],
    ["--cidr=2001:db8::/32,0.0.0.0/0"],
    ["--cidr=[2001:db8::1]/64"],
    ["--port"],
    ["--port", "--nonip"],
    ["--mac=00:1f:f3:3c:e1:13,0a:0b:0c:0d:0e:0f"],
    ["--mac=zz:1f,0a:0b:0c:0d:0e:0f", "--reverse"],
    ["--mac=00:1f:f3:3c:e1:13", "--include=P:3-9,200-"],
    ["--cidr=96.17.211.0/24", "--exclude=P:0-40,77-"],
    ["--cidr=96.17.211.0/24", "--include=E:96.0.0.0/8,10.1.0.0/16"],
    ["--cidr=96.17.211.0/24", "--exclude=B:96.0.0.0/8"],
    ["--port", "--exclude=S:96.17.211.0/24"],
    ["--comment=gpu", "--port"],
    ["--auto=bridge"],
    ["--auto=client", "--ratio=0.5"],
    ["--auto=server", "--nonip"],
    ["--auto=first", "--ratio=0"],
    ["--auto=router", "--nonip", "--minmask=24", "--maxmask=16"],
    ["--regex=96.17.211.*"],
    ["--regex=^(10|96)\\.[0-9]+", "--reverse"],
    ["--regex=::", "--nonip"],
    ["--regex=[a-f]:[0-9]|^0\\.", "--include=P:3-90"],
]


def _both(pcap, args):
    """GPU and oracle results, or the fact that both refused (packet2tree's len_error)."""
    try:
        exp = oracle_lib.tcpprep(pcap, args)
    except ValueError:
        exp = "error"
    try:
        got = TP.cache(pcap, args)
    except RuntimeError as e:
        assert "too small to process" in str(e)
        got = "error"
    return got, exp


@pytest.mark.parametrize("line", range(len(OPTION_LINES)))
def test_gpu_matches_oracle_adversarial(line):
    pcap = _adversarial()
    args = OPTION_LINES[line]
    got, exp = _both(pcap, args)
    assert got == exp


@pytest.mark.parametrize("mode", ["bridge", "client", "server", "first", "router"])
def test_gpu_auto_matches_oracle_without_short_tcp(mode):
    """the adversarial corpus minus the records that make packet2tree abort (a TCP header
    short of its captured bytes, after the reader's trim or behind a mutated IHL): each kept
    record passes the oracle's first pass on its own"""
    def alone_ok(r):
        try:
            oracle_lib.tcpprep(synth.build_pcap([r]), ["--auto=bridge"])
            return True
        except ValueError:
            return False
    recs = [r for r in synth.records(_adversarial(seed=11)) if min(r[2], r[3]) >= 74 and alone_ok(r)]
    pcap = synth.build_pcap(recs)
    got, exp = _both(pcap, [f"--auto={mode}"])
    assert got == exp and got != "error"


def test_gpu_auto_reports_len_error_like_the_reference():
    recs = synth.records(T.test_pcap())[:20]
    d = bytearray(recs[3][4][:40])  # an IPv4/TCP frame cut inside its TCP header
    d[12:14], d[14], d[23] = (0x08, 0x00), 0x45, 6
    recs[3] = (0, 0, 40, 40, bytes(d))
    pcap = synth.build_pcap(recs)
    assert _both(pcap, ["--auto=bridge"]) == ("error", "error")


@pytest.mark.parametrize("zc,zl", [(0, 0), (0, 60), (60, 0), (60, 300_000)])
@pytest.mark.parametrize("args", [["--port"], ["--cidr=96.17.211.0/24", "--include=P:3-90"], ["--auto=bridge"],
                                  ["--mac=00:1f:f3:3c:e1:13"]])
def test_reader_exit_writes_no_cache(zc, zl, args):
    """safe_pcap_next (tcpprep.c:353 -> src/common/utils.c:136-156) exit(-1)s at a record with
    a zero len or caplen or len > MAX_SNAPLEN, before write_cache (tcpprep.c:194): no cache,
    on the GPU as in the oracle -- and the records before it do not matter"""
    recs = synth.records(T.test_pcap())
    ts, tu, cl, ln, d = recs[50]
    recs[50] = (ts, tu, zc, zl, d[:zc])
    pcap = synth.build_pcap(recs)
    with pytest.raises(ValueError):
        oracle_lib.tcpprep(pcap, args)
    with pytest.raises(RuntimeError, match="safe_pcap_next"):
        TP.cache(pcap, args)


def test_gpu_matches_oracle_full_size_imix():
    pcap = synth.pcap_imix(500_000, seed=3)
    for args in (["--port"], ["--cidr=10.0.0.0/9,172.16.128.0/17", "--reverse"], ["--auto=bridge"],
                 ["--auto=first"]):
        assert TP.cache(pcap, args) == oracle_lib.tcpprep(pcap, args)


def test_gpu_matches_oracle_v4v6():
    pcap = synth.pcap_mixed_v4v6(100_000, seed=5)
    for args in (["--port"], ["--cidr=10.0.0.0/8"], ["--mac=00:66:77:88:99:aa", "--include=E:172.16.0.0/12"]):
        assert TP.cache(pcap, args) == oracle_lib.tcpprep(pcap, args)


def test_gpu_cache_drives_tcprewrite():
    """the cache it writes is read back by the GPU tcprewrite path (-c)."""
    import tcpreplay_amd as TA
    c = TP.cache(T.test_pcap(), T.args("cidr"))
    args = ["--endpoints=10.10.0.1:10.10.0.2", "--fixcsum"]
    te = TA.TcpEdit(args)
    rc, out = te.rewrite(T.test_pcap(), cache=c)
    orc, oout = oracle_lib.rewrite(T.test_pcap(), args, cache=c)
    assert rc == orc and out == oout


def test_mac_mode_short_records_get_no_entry():
    recs = synth.records(T.test_pcap())[:9]
    recs.insert(4, (0, 0, 10, 10, bytes(10)))
    pcap = synth.build_pcap(recs)
    # record 5 is 10 bytes long: no entry, unless the packet list turns it into DONT_SEND first
    for extra, body in (([], "babb03"), (["--exclude=P:6"], "bab803"), (["--exclude=P:5"], "baec0e")):
        args = ["--no-arg-comment", "--mac=00:1f:f3:3c:e1:13"] + extra
        c = TP.cache(pcap, args)
        assert c == oracle_lib.tcpprep(pcap, args)
        assert int.from_bytes(c[12:20], "big") == 10 and c[24:].hex() == body


def test_rejects_unsupported_modes_loudly():
    for args in (["--auto=bogus"], ["--auto=router", "--minmask=8", "--maxmask=16"], ["--regex=(96"], ["--port", "--include=F:tcp"], []):
        with pytest.raises(ValueError):
            TP.TcpPrep(args)


def test_tcpprep_tool_file_to_file(tmp_path):
    """bin/tcpprep against the reference's own cache files (test/Makefile.am:87-104)"""
    import os
    import subprocess
    import tcpreplay_amd as TA
    tool = os.path.join(os.path.dirname(TA.LIB_PATH), "..", "bin", "tcpprep")
    src = os.path.join(T.GOLDEN, "test.pcap")
    for name in ("auto_router", "cidr_reverse", "include_packets", "comment"):
        out = tmp_path / ("prep." + name)
        subprocess.run([tool, "-i", src, "-o", str(out)] + T.args(name), check=True, timeout=60)
        assert out.read_bytes() == T.golden(name)


def test_gpu_services_file_matches_oracle(tmp_path):
    from test_tcpprep_oracle import SERVICES
    f = tmp_path / "services"
    f.write_text(SERVICES)
    for pcap in (T.test_pcap(), _adversarial(), synth.pcap_imix(200_000, seed=4)):
        args = ["--no-arg-comment", "--port", f"--services={f}"]
        assert TP.cache(pcap, args) == oracle_lib.tcpprep(pcap, args)


@pytest.mark.parametrize("pattern", ["::", "^::ffff:", r"^::[0-9]+\.", ":0:", "^[0-9a-f]{1,4}:[0-9a-f]{1,4}::",
                                     r"\.(1|2)[0-9]$", "^fe80", "^[^:]+$", "(::|:0:)[1-9a-f]"])
def test_regex_over_every_ipv6_text_shape(pattern):
    """inet_ntop's IPv6 forms, as the device prints them through the DFA: the first
    longest zero run compressed (or none shorter than 2 words), IPv4-compatible and
    -mapped tails in dotted form, leading-zero-free lowercase hex; IPv4 sources too"""
    rng = np.random.default_rng(5)
    v6 = synth.records(synth.pcap_fixed(3000, 90, ipv6=True, seed=3))
    v4 = synth.records(synth.pcap_fixed(500, 64, seed=4))
    recs = []
    for i, (ts, tu, cl, ln, d) in enumerate(v6):
        d = bytearray(d)
        w = [int(x) for x in rng.choice([0, 0, 0, 1, 0xffff, 0xfe80, int(rng.integers(0, 65536))], size=8)]
        if i % 7 == 0:
            w[:6] = [0, 0, 0, 0, 0, 0xffff if i % 14 else 0]
        d[22:38] = b"".join(x.to_bytes(2, "big") for x in w)
        recs.append((ts, tu, cl, ln, bytes(d)))
    recs += v4
    pcap = synth.build_pcap(recs)
    args = ["--no-arg-comment", "--regex=" + pattern]
    assert TP.cache(pcap, args) == oracle_lib.tcpprep(pcap, args)


AUTO_FILTERS = [["--include=P:5-60"], ["--exclude=P:1-9,30-31,100-"], ["--include=S:172.16.0.0/12"],
                ["--exclude=D:10.0.0.0/8"], ["--include=B:0.0.0.0/0"], ["--exclude=E:96.17.211.0/24"]]


@pytest.mark.parametrize("mode", ["bridge", "client", "server", "first", "router"])
@pytest.mark.parametrize("filt", range(len(AUTO_FILTERS)))
def test_gpu_auto_with_include_exclude(mode, filt):
    """--auto with --include/--exclude (tcpprep.c:362-375, 413-428 in both passes): the first
    pass's DONT_SEND entries of the filtered records, then every record's entry -- GPU ==
    oracle, on the reference's test.pcap and on an IMIX capture"""
    args = ["--no-arg-comment", f"--auto={mode}"] + AUTO_FILTERS[filt]
    for pcap in (T.test_pcap(), synth.pcap_imix(3000, seed=filt)):
        got, exp = _both(pcap, args)
        assert got == exp and got != "error"


def test_gpu_auto_filter_buffer_size_message_is_the_size_needed():
    """--auto with a filter: the cache can hold a first-pass entry per filtered record before
    the body, so tcpprep_cache_pcap needs hdr + (2n + 3) / 4 bytes -- and a too-small buffer's
    error names that size, which then succeeds"""
    import ctypes
    import re
    pcap = synth.pcap_imix(3000, seed=3)
    p = TP.TcpPrep(["--no-arg-comment", "--auto=bridge", "--exclude=P:1-9,30-31,100-"])
    try:
        L = p._L
        small = ctypes.create_string_buffer(24 + (3000 + 3) // 4)
        assert L.tcpprep_cache_pcap(p._ctx, pcap, len(pcap), small, len(small)) < 0
        m = re.search(r"too small \((\d+) < (\d+)\)", p.geterr())
        need = int(m.group(2))
        assert need == 24 + (2 * 3000 + 3) // 4
        buf = ctypes.create_string_buffer(need)
        n = L.tcpprep_cache_pcap(p._ctx, pcap, len(pcap), buf, need)
        assert n > 0 and buf.raw[:n] == p.cache(pcap)
    finally:
        p.close()
