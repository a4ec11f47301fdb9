"""GPU parity: the HIP path (through the C-ABI) against the reference goldens and
the CPU oracle.  Integer/byte work, so every comparison is bit-exact."""
import os
import random
import struct

import numpy as np
import pytest

import golden_cases as G
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C2_ARGS = ["--seed=42", "--fixcsum"]
C3_ARGS = ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]
C4_ARGS = ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
           "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add", "--enet-vlan-tag=45",
           "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"]
C5_ARGS = ["--fixcsum"]


def gpu_rewrite(pcap, args, cache=None, with_status=False):
    te = TA.TcpEdit(args)
    try:
        return te.rewrite(pcap, cache, with_status=with_status)
    finally:
        te.close()


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i
    return n


def assert_same(out, exp):
    assert len(out) == len(exp) and out == exp, f"first difference at byte {first_diff(out, exp)}"


# ---------------------------------------------------------------- goldens
@pytest.mark.parametrize("case", G.IN_SCOPE, ids=[c[0] for c in G.IN_SCOPE])
def test_gpu_matches_reference_golden(built, case):
    name, inp, cache, args, _ = case
    rc, out = gpu_rewrite(G.read(inp), args, G.read(cache) if cache else None)
    assert rc == 0
    assert_same(out, G.read(name))


# ---------------------------------------------------------------- BASELINE configs vs oracle
@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C5"])
def test_gpu_matches_oracle_on_baseline_configs(built, cfg):
    cache = None
    if cfg == "C2":
        pcap, args = S.pcap_fixed(100_000, 64, seed=2), C2_ARGS
    elif cfg == "C3":
        pcap, args = S.pcap_imix(60_000, seed=3), C3_ARGS
    elif cfg == "C4":
        pcap, args = S.pcap_imix(60_000, seed=4), C4_ARGS
        cache = S.tcpprep_cache(60_000, seed=4, nosend_every=97)
    else:
        pcap, args = S.pcap_mixed_v4v6(20_000, 1514, seed=5), C5_ARGS
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out = gpu_rewrite(pcap, args, cache)
    assert rc == rc_o == 0
    assert_same(out, exp)


def test_fixcsum_is_idempotent_and_valid(built):
    pcap = S.pcap_imix(50_000, seed=9)
    # corrupt every 7th IPv4 header checksum; --fixcsum must restore the original bytes
    b = bytearray(pcap)
    for i, off in enumerate(record_offsets(pcap)):
        if i % 7 == 0:
            b[off + 16 + 24] ^= 0x5A
    rc, out = gpu_rewrite(bytes(b), ["--fixcsum"])
    assert rc == 0
    assert_same(out, pcap)
    rc, out2 = gpu_rewrite(out, ["--fixcsum"])
    assert_same(out2, out)


def record_offsets(pcap):
    offs, off = [], 24
    while off + 16 <= len(pcap):
        offs.append(off)
        off += 16 + struct.unpack_from("<I", pcap, off + 8)[0]
    return offs


# ---------------------------------------------------------------- differential fuzzing vs oracle
OPTION_POOL = [c[3] for c in G.IN_SCOPE if c[2] is None] + [
    ["--fixcsum", "--efcs"], ["--seed=7", "--skipbroadcast", "--fixcsum"], ["--ttl=+3", "--tos=7"],
    ["--enet-vlan=del", "--fixcsum"], ["--fixlen=pad", "--fixcsum"], ["--mtu-trunc", "--mtu=100", "--fixcsum"],
    ["--srcipmap=0.0.0.0/0:10.1.0.0/16", "--dstipmap=96.0.0.0/8:11.0.0.0/8", "--fixcsum"],
    ["--pnat=[::/0]:[2001:db8:aaaa::/40]", "--fixcsum"], ["--tclass=12", "--flowlabel=4660", "--ttl=9"],
    ["--portmap=1-65535:7", "--tcp-sequence=5"], ["--fixhdrlen", "--fixcsum"], ["--skip-soft-errors", "--seed=3"],
    # non-octet IPv6 masks: remap_ipv6's stray write on the generic lane
    ["--pnat=[::/0]:[2001:db8:aaaa::/36]", "--fixcsum"], ["--srcipmap=[::/0]:[2001:db8::/20]", "--seed=5"],
    ["--pnat=10.0.0.0/8:192.168.0.0/20,[::/0]:[fd00::/9]"],
    # the hdlc encoder's fallback fields on Ethernet: a tagged frame's vlan flag (1), else a
    # soft error written half-moved (hdlc.c:240-288)
    ["--dlt=hdlc"], ["--dlt=hdlc", "--hdlc-control=9", "--fixcsum"],
]


def mutate(recs, rng, reader_stop=None):
    """random header bytes, snaplen truncation (len > caplen), len < caplen (the reader's
    safe_pcap_next trims caplen to len, src/common/utils.c:159-162) and VLAN/QinQ/MPLS
    insertion.  reader_stop = "len" / "cap" / "both": one record near the end gets len 0,
    caplen 0 or both -- safe_pcap_next's exit (utils.c:147-156): the output ends before it"""
    out = []
    for ts, tu, cl, ln, data in recs:
        d = bytearray(data)
        r = rng.random()
        if r < 0.25 and len(d) > 14:  # random header byte
            i = rng.randrange(0, min(len(d), 80))
            d[i] = rng.randrange(256)
        elif r < 0.32 and cl > 1:  # snaplen-truncated capture
            cl = rng.randrange(1, cl + 1)
            d = d[:cl]
        elif r < 0.36:  # len > caplen
            ln = cl + rng.randrange(0, 100)
        elif r < 0.40 and cl > 1:  # len < caplen: the record is read as len bytes
            ln = rng.choice([rng.randrange(1, cl), max(1, cl - 4), max(1, cl - rng.randrange(1, 30))])
        elif r < 0.46 and len(d) > 14:  # 802.1Q / QinQ / MPLS encapsulations
            tag = rng.choice([b"\x81\x00", b"\x88\xa8", b"\x91\x00"])
            d = d[:12] + tag + bytes([rng.randrange(256), rng.randrange(256)]) + d[12:]
            cl, ln = len(d), ln + 4
        out.append((ts, tu, cl, ln, bytes(d)))
    if reader_stop and len(out) > 4:
        k = len(out) - rng.randrange(2, 5)
        ts, tu, cl, ln, d = out[k]
        if reader_stop in ("cap", "both"):
            cl, d = 0, b""
        if reader_stop in ("len", "both"):
            ln = 0
        out[k] = (ts, tu, cl, ln, d)
    return out


@pytest.mark.parametrize("seed", range(24))
def test_gpu_matches_oracle_on_mutated_captures(built, seed):
    rng = random.Random(seed)
    recs = mutate(S.records(G.read("test.pcap")), rng, reader_stop=[None, None, None, "len", "cap", "both"][seed % 6])
    pcap = S.build_pcap(recs)
    args = OPTION_POOL[seed % len(OPTION_POOL)]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, st = gpu_rewrite(pcap, args, with_status=True)
    assert not (st & TA.ST.UNSUPPORTED).any()  # stale-buffer reads (Q8) are replayed, not refused
    assert rc == rc_o
    assert_same(out, exp)


# ---------------------------------------------------------------- per-packet API
@pytest.mark.parametrize("args", [["--fixcsum"], ["--seed=55"], ["--enet-vlan=add", "--enet-vlan-tag=45"]])
def test_tcpedit_packet_api(built, args):
    recs = S.records(G.read("test.pcap"))[:40]
    _, exp = O.rewrite(S.build_pcap(recs), args)
    exp_recs = S.records(exp)
    te = TA.TcpEdit(args)
    got = []
    for ts, tu, cl, ln, data in recs:
        buf = bytearray(262166)
        buf[:cl] = data
        rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf)
        assert rc != TA.TCPEDIT_ERROR
        got.append((ts, tu, h["caplen"], h["len"], bytes(buf[:h["caplen"]])))
    te.close()
    assert got == exp_recs


def _per_packet(te, recs, bufsize=262166):
    L = TA.load()
    got = []
    for ts, tu, cl, ln, data in recs:
        buf = bytearray(bufsize)
        buf[:cl] = data
        rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf)
        got.append((rc, h["caplen"], h["len"], bytes(buf[:h["caplen"]]) if rc != TA.TCPEDIT_ERROR else b""))
    return got, (L.tcpedit_get_pkts_edited(te._ctx), L.tcpedit_get_total_bytes(te._ctx))


def _launch_path(fn):
    """run fn() with tcpedit_packet's launch-per-call path (no resident server)"""
    old = os.environ.get("TCPEDIT_HIP_PACKET_SERVER")
    os.environ["TCPEDIT_HIP_PACKET_SERVER"] = "0"
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop("TCPEDIT_HIP_PACKET_SERVER", None)
        else:
            os.environ["TCPEDIT_HIP_PACKET_SERVER"] = old


@pytest.mark.parametrize("k", range(len(OPTION_POOL)))
def test_packet_server_matches_the_launch_path(built, k):
    """the resident server (te_packet_server) edits every record as the launch-per-call
    path does: status, header, bytes and the context's counters"""
    args = OPTION_POOL[k]
    recs = mutate(S.records(G.read("test.pcap")), random.Random(100 + k))
    te = TA.TcpEdit(args)
    try:
        got = _per_packet(te, recs)
    finally:
        te.close()
    te = TA.TcpEdit(args)
    try:
        exp = _launch_path(lambda: _per_packet(te, recs))
    finally:
        te.close()
    assert got[1] == exp[1]
    for i, (a, b) in enumerate(zip(got[0], exp[0])):
        assert a == b, f"record {i}"


def test_packet_server_relaunches_after_idle_and_serves_two_contexts(built):
    """the server leaves after 50 ms without a request and the next call launches it
    again; two contexts keep a server each"""
    import time
    recs = S.records(G.read("test.pcap"))[:12]
    pcap = S.build_pcap(recs)
    a1, a2 = ["--seed=9", "--fixcsum"], ["--enet-vlan=add", "--enet-vlan-tag=3"]
    exp1, exp2 = S.records(O.rewrite(pcap, a1)[1]), S.records(O.rewrite(pcap, a2)[1])
    t1, t2 = TA.TcpEdit(a1), TA.TcpEdit(a2)
    try:
        for i, (ts, tu, cl, ln, data) in enumerate(recs):
            for te, exp in ((t1, exp1), (t2, exp2)):
                buf = bytearray(262166)
                buf[:cl] = data
                rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf)
                assert rc != TA.TCPEDIT_ERROR
                assert (ts, tu, h["caplen"], h["len"], bytes(buf[:h["caplen"]])) == exp[i]
            if i % 4 == 3:
                time.sleep(0.12)
    finally:
        t1.close()
        t2.close()


def test_packet_server_that_never_answers_ends_bounded(built, tmp_path):
    """a server that stops answering (forced: TCPEDIT_HIP_SRV_TEST_STUCK) is stopped with a
    bounded wait and never stream-synced: the call falls back to the launch path with the
    same bytes, and tcpedit_close and the process exit do not hang"""
    import subprocess
    import sys
    script = tmp_path / "stuck.py"
    script.write_text(
        "import sys\n"
        f"sys.path[:0] = [{ROOT!r}, {os.path.join(ROOT, 'tests')!r}]\n"
        "import golden_cases as G, oracle_lib as O, tcpreplay_amd as TA\n"
        "from tcpreplay_amd import synth as S\n"
        "recs = S.records(G.read('test.pcap'))[:6]\n"
        "exp = S.records(O.rewrite(S.build_pcap(recs), ['--seed=3'])[1])\n"
        "te = TA.TcpEdit(['--seed=3'])\n"
        "for i, (ts, tu, cl, ln, d) in enumerate(recs):\n"
        "    buf = bytearray(262166); buf[:cl] = d\n"
        "    rc, h = te.packet({'ts_sec': ts, 'ts_usec': tu, 'caplen': cl, 'len': ln}, buf)\n"
        "    assert (ts, tu, h['caplen'], h['len'], bytes(buf[:h['caplen']])) == exp[i], i\n"
        "te.close()\n"
        "print('ok')\n")
    env = dict(os.environ, TCPEDIT_HIP_SRV_TEST_STUCK="1")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, timeout=100, env=env)
    assert r.returncode == 0 and b"ok" in r.stdout, r.stderr.decode()[-2000:]
    # waited for once: a stuck server's later stops return at once
    assert r.stderr.count(b"did not leave") == 1


def test_packet_server_declines_records_larger_than_its_slot(built):
    """a record past the block's LDS slot goes the launch-per-call way (same bytes)"""
    rng = random.Random(7)
    recs = S.records(S.pcap_fixed(4, 1400, seed=8))
    big = []
    for ts, tu, cl, ln, d in recs:
        d = d + bytes(rng.randrange(256) for _ in range(40000))
        big.append((ts, tu, len(d), len(d), d))
    pcap = S.build_pcap(big + recs)
    _, exp = O.rewrite(pcap, ["--ttl=4"])
    te = TA.TcpEdit(["--ttl=4"])
    try:
        got, _ = _per_packet(te, big + recs)
    finally:
        te.close()
    assert [(g[1], g[2], g[3]) for g in got] == [(e[2], e[3], e[4]) for e in S.records(exp)]


@pytest.mark.parametrize("opt", ["srcipmap", "dstipmap", "pnat", "pnat2", "endpoints_v6"])
def test_cidr_maps_past_the_inline_list(built, opt):
    """CIDR maps longer than the config's 16 inline pairs: the rest from the spill list in
    HBM, in the reference's first-match order (cidr.c:290-418)"""
    pairs = [f"10.{i}.0.0/16:172.{16 + i % 16}.{i}.0/24" for i in range(37)]
    pairs.append("0.0.0.0/0:198.51.100.0/24")  # the catch-all past the inline list
    lst = ",".join(pairs)
    if opt == "pnat2":
        args = [f"--pnat={lst}", "--pnat=" + ",".join(reversed(pairs)), "--fixcsum"]
    elif opt == "endpoints_v6":
        v6 = ",".join(f"[2001:db8:{i:x}::/48]:[fd00:{i:x}::/48]" for i in range(30)) + ",[::/0]:[fd99::/64]"
        args = [f"--pnat={lst},{v6}", "--fixcsum"]
    else:
        args = [f"--{opt}={lst}", "--fixcsum"]
    rng = np.random.default_rng(5)
    pcap = S.pcap_imix(4000, seed=11)
    recs = S.records(pcap)
    out_recs = []
    for k, (ts, tu, cl, ln, d) in enumerate(recs):  # addresses spread over the 40 prefixes
        d = bytearray(d)
        if d[12:14] == b"\x08\x00":
            d[26:28] = bytes([10, int(rng.integers(0, 45))])
            d[30:32] = bytes([10, int(rng.integers(0, 45))])
        out_recs.append((ts, tu, cl, ln, bytes(d)))
    pcap = S.build_pcap(out_recs)
    pcap = pcap + S.pcap_mixed_v4v6(200, 200, seed=3)[24:]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = gpu_rewrite(pcap, args)
    assert rc == rc_o == 0
    assert_same(out, exp)


# ---------------------------------------------------------------- edge cases
def test_empty_capture(built):
    hdr = G.read("test.pcap")[:24]
    rc, out = gpu_rewrite(hdr, ["--fixcsum"])
    rc_o, exp = O.rewrite(hdr, ["--fixcsum"])
    assert rc == rc_o == 0
    assert_same(out, exp)


def test_hard_error_truncates_output(built):
    recs = S.records(G.read("test.pcap"))[:10]
    ts, tu, cl, ln, d = recs[2]
    d = bytearray(d)
    assert d[12:14] == b"\x08\x00"
    d[14] = 0x55  # IP version 5 with ethertype IPv4 -> TCPEDIT_ERROR (edit_packet.c:73-79)
    recs[2] = (ts, tu, cl, ln, bytes(d))
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, ["--fixcsum"])
    rc, out = gpu_rewrite(pcap, ["--fixcsum"])
    assert rc_o == -1 and rc == TA.TCPEDIT_ERROR
    assert_same(out, exp)
    assert len(S.records(out)) == 2


def test_stale_buffer_dependency_is_replayed(built):
    # IPv6/UDP whose payload length overstates the captured bytes: the reference's
    # checksum then reads its static buffer past caplen; the device replays
    # the buffer and writes the reference's checksum
    pcap = S.pcap_fixed(4, 200, ipv6=True, proto=17)
    recs = S.records(pcap)
    ts, tu, cl, ln, d = recs[3]
    d = bytearray(d)
    struct.pack_into(">H", d, 18, 146 + 50)
    recs[3] = (ts, tu, cl, ln, bytes(d))
    pcap = S.build_pcap(recs)
    te = TA.TcpEdit(["--fixcsum"])
    b = TA.Batch(te, pcap)
    assert b.run() == TA.TCPEDIT_OK
    r = b.result()
    assert r.unsupported == 0 and r.stale_records == 1 and r.first_unsupported == -1
    assert_same(b.output(), O.rewrite(pcap, ["--fixcsum"])[1])
    b.close()
    te.close()


@pytest.mark.parametrize("args", [["--fixcsum"], ["--seed=42", "--fixcsum"], ["--enet-vlan=add", "--enet-vlan-tag=3"]])
def test_huge_records_use_the_hbm_slot_path(built, args):
    small = S.records(S.pcap_fixed(3, 64, seed=1))
    big = S.records(S.pcap_fixed(2, 100_000, seed=2)) + S.records(S.pcap_fixed(1, 262_000, seed=3, ipv6=True))
    recs = [small[0], big[0], small[1], big[1], big[2], small[2]]
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = gpu_rewrite(pcap, args)
    assert rc == rc_o == 0
    assert_same(out, exp)


@pytest.mark.parametrize("args", [["--fixcsum"], ["--mtu-trunc", "--mtu=262000", "--fixcsum"],
                                  ["--enet-subsmac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee", "--fixcsum"],
                                  ["--fuzz-seed=3", "--fuzz-factor=1", "--fixcsum"]])
def test_checksum_reads_flush_against_buffer_ends(built, args):
    """csum_bytes reads whole aligned 16-byte quads: each holds at least one of the packet's
    bytes, so no read leaves the granule of a byte it owns.  Records placed flush against
    the end of every buffer the generic lane sums in -- the input image (last record ends
    the capture, at every residue mod 16), a huge record's HBM scratch slot (> 36 KiB
    records, odd sizes, IPv4 and IPv6) and the last LDS tile -- must equal the oracle."""
    for tail, v6, proto in [(100_001, True, 17), (100_013, False, 6), (65_535, True, 6), (262_143, False, 17),
                            (1_514, False, 17), (1_513, True, 6), (61, False, 17), (77, False, 6), (95, True, 17)]:
        recs = S.records(S.pcap_imix(300, seed=tail % 97))
        recs += S.records(S.pcap_fixed(1, tail, seed=tail % 13, ipv6=v6, proto=proto))
        pcap = S.build_pcap(recs)
        rc_o, exp = O.rewrite(pcap, args)
        rc, out = gpu_rewrite(pcap, args)
        assert rc == rc_o == 0, (tail, args)
        assert_same(out, exp)


def test_nanosecond_capture_is_written_in_microseconds(built):
    p = bytearray(G.read("test.pcap"))
    p[0:4] = struct.pack("<I", 0xA1B23C4D)
    for off in record_offsets(bytes(p)):
        us = struct.unpack_from("<I", p, off + 4)[0]
        struct.pack_into("<I", p, off + 4, us * 1000 + 999)
    rc, out = gpu_rewrite(bytes(p), ["--fixcsum"])
    assert rc == 0
    assert_same(out, G.read("test2.rewrite_fixcsum"))


@pytest.mark.slow
def test_full_size_c2_matches_oracle(built):
    pcap = S.pcap_fixed(1_000_000, 64, seed=1)
    rc_o, exp = O.rewrite(pcap, C2_ARGS)
    rc, out = gpu_rewrite(pcap, C2_ARGS)
    assert rc == rc_o == 0
    assert_same(out, exp)


# ---------------------------------------------------------------- pipelined whole-file path
def pipe_rewrite(pcap, args, cache=None, chunk=1 << 20):
    te = TA.TcpEdit(args)
    try:
        return te.rewrite_pipelined(pcap, cache, chunk_bytes=chunk)
    finally:
        te.close()


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C5"])
def test_pipelined_matches_oracle_on_baseline_configs(built, cfg):
    """Several 1 MiB chunks per capture: record boundaries, cache lookups (pkt_base) and
    output placement across chunks."""
    cache = None
    if cfg == "C2":
        pcap, args = S.pcap_fixed(60_000, 64, seed=12), C2_ARGS
    elif cfg == "C3":
        pcap, args = S.pcap_imix(20_000, seed=13), C3_ARGS
    elif cfg == "C4":
        pcap, args = S.pcap_imix(20_000, seed=14), C4_ARGS
        cache = S.tcpprep_cache(20_000, seed=14, nosend_every=97)
    else:
        pcap, args = S.pcap_mixed_v4v6(4_000, 1514, seed=15), C5_ARGS
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out = pipe_rewrite(pcap, args, cache)
    assert rc == rc_o == 0
    assert_same(out, exp)


@pytest.mark.parametrize("case", G.IN_SCOPE[:6], ids=[c[0] for c in G.IN_SCOPE[:6]])
def test_pipelined_matches_reference_golden(built, case):
    name, inp, cache, args, _ = case
    rc, out = pipe_rewrite(G.read(inp), args, G.read(cache) if cache else None)
    assert rc == 0
    assert_same(out, G.read(name))


def test_pipelined_context_reuse_and_edge_cases(built):
    args = ["--seed=5", "--fixcsum"]
    te = TA.TcpEdit(args)
    try:
        # the empty capture, then a capture ending in a truncated record, then a big one
        empty = S.build_pcap([])
        rc, out = te.rewrite_pipelined(empty, chunk_bytes=1 << 20)
        assert rc == 0 and out == O.rewrite(empty, args)[1]
        big = S.pcap_imix(30_000, seed=16)
        cut = big[: len(big) - 700]  # the last record is cut short: libpcap stops before it
        for img in (cut, big, big):
            rc_o, exp = O.rewrite(img, args)
            rc, out = te.rewrite_pipelined(img, chunk_bytes=1 << 20)
            assert rc == rc_o == 0
            assert_same(out, exp)
        # the same slots with the default chunk size
        rc, out = te.rewrite_pipelined(big)
        assert rc == 0 and out == O.rewrite(big, args)[1]
    finally:
        te.close()


@pytest.mark.parametrize("zc,zl", [(64, 300_000), (0, 0), (0, 64), (64, 0)])
def test_pipelined_hard_error_truncates_in_a_later_chunk(built, zc, zl):
    """len > MAX_SNAPLEN, a zero len or caplen: safe_pcap_next exit(-1)s (src/common/
    utils.c:136-156), the output keeps the earlier chunks' and this chunk's earlier records"""
    recs = S.records(S.pcap_fixed(40_000, 64, seed=17))
    ts, tu, cl, ln, d = recs[30_000]
    recs[30_000] = (ts, tu, zc, zl, d[:zc])
    pcap = S.build_pcap(recs)
    args = ["--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = pipe_rewrite(pcap, args)
    assert rc == rc_o == -1
    assert_same(out, exp)


@pytest.mark.parametrize("args", [["--fixcsum"], ["--seed=42", "--fixcsum"],
                                  ["--enet-vlan=add", "--enet-vlan-tag=45", "--fixcsum"], ["--efcs"]])
def test_pipelined_and_batch_trim_caplen_to_len(built, args):
    """len < caplen records spread over the chunks: safe_pcap_next trims caplen to len
    (src/common/utils.c:159-162), so the output shrinks where they are (scan placement)"""
    recs = S.records(S.pcap_imix(60_000, seed=19))
    for i in range(11, len(recs), 997):
        ts, tu, cl, ln, d = recs[i]
        recs[i] = (ts, tu, cl, max(1, cl - 1 - i % 300), d)
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = pipe_rewrite(pcap, args)
    assert rc == rc_o == 0
    assert_same(out, exp)
    rc, out = gpu_rewrite(pcap, args)
    assert rc == 0
    assert_same(out, exp)


@pytest.mark.parametrize("mode", [[], ["--pipeline=1"]])
def test_tcprewrite_tool_file_to_file(built, tmp_path, mode):
    """bin/tcprewrite, batch and pipelined modes, against the reference's own goldens
    (config 1: --fixcsum; the tcpprep-cache endpoint/VLAN chain)."""
    import subprocess
    tool = os.path.join(os.path.dirname(TA.LIB_PATH), "..", "bin", "tcprewrite")
    for name in ("test2.rewrite_fixcsum", "test2.rewrite_endpoint"):
        case = next(c for c in G.CASES if c[0] == name)
        out = tmp_path / f"{name}.out"
        cmd = [tool, "-i", os.path.join(G.GOLDEN_DIR, case[1]), "-o", str(out)] + case[3] + mode
        if case[2]:
            cmd += ["-c", os.path.join(G.GOLDEN_DIR, case[2])]
        subprocess.run(cmd, check=True, capture_output=True, timeout=60)
        assert_same(out.read_bytes(), G.read(name))


# ---------------------------------------------------------------- VLAN add: static +4 placement
def test_vlan_add_static_grow_matches_oracle_and_scan(built, monkeypatch):
    """--enet-vlan=add places record i at its input offset + 4 i (no scan); the same
    capture placed by scan + look-back (TCPEDIT_HIP_NO_GROW) and the oracle agree."""
    pcap = S.pcap_imix(30_000, seed=11)
    cache = S.tcpprep_cache(30_000, seed=3)
    _, exp = O.rewrite(pcap, C4_ARGS, cache)
    rc, out = gpu_rewrite(pcap, C4_ARGS, cache)
    assert rc == 0
    assert_same(out, exp)
    monkeypatch.setenv("TCPEDIT_HIP_NO_GROW", "1")
    rc, out2 = gpu_rewrite(pcap, C4_ARGS, cache)
    assert rc == 0
    assert_same(out2, exp)


def test_vlan_add_unedited_records_fall_back_to_scan(built):
    """Records the tcpprep cache marks NOSEND are written unedited (no VLAN tag, no +4):
    the static placement sees them, and the batch is placed again by scan -- on every
    run of the same batch."""
    n = 20_000
    pcap = S.pcap_imix(n, seed=12)
    cache = S.tcpprep_cache(n, seed=4, nosend_every=97)
    _, exp = O.rewrite(pcap, C4_ARGS, cache)
    te = TA.TcpEdit(C4_ARGS)
    try:
        b = TA.Batch(te, pcap, cache)
        for _ in range(3):
            assert b.run() == 0
            assert_same(b.output(), exp)
        b.close()
    finally:
        te.close()


def test_vlan_add_hard_error_truncates_at_static_offset(built):
    """A hard error under VLAN add ends the output at that record's statically placed
    offset (+4 per earlier record), as the oracle does."""
    recs = S.records(S.pcap_imix(2_000, seed=13))
    ts, tu, cl, ln, d = recs[1_234]
    d = bytearray(d)
    assert d[12:14] == b"\x08\x00"
    d[14] = 0x55  # IP version 5 with ethertype IPv4 -> TCPEDIT_ERROR (edit_packet.c:73-79)
    recs[1_234] = (ts, tu, cl, ln, bytes(d))
    pcap = S.build_pcap(recs)
    args = ["--enet-vlan=add", "--enet-vlan-tag=7", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = gpu_rewrite(pcap, args)
    assert rc_o == -1 and rc == TA.TCPEDIT_ERROR
    assert_same(out, exp)
    assert len(S.records(out)) == 1_234


def _mixed_sizes_pcap(seed):
    """IPv4/IPv6 x UDP/TCP records of assorted sizes (odd ones too), interleaved"""
    rng = random.Random(seed)
    parts = []
    for size, v6, proto in [(42, False, 17), (61, False, 17), (64, False, 6), (77, False, 6), (79, False, 17),
                            (90, True, 17), (97, True, 6), (333, False, 6), (1514, True, 17), (65, False, 17)]:
        parts += S.records(S.pcap_fixed(300, size, seed=rng.randrange(1 << 20), ipv6=v6, proto=proto))
    rng.shuffle(parts)
    return S.build_pcap(parts)


@pytest.mark.parametrize("args", [
    ["--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"],
    ["--enet-vlan=add", "--enet-vlan-tag=4095", "--enet-vlan-proto=802.1ad", "--seed=9", "--fixcsum"],
    ["--enet-vlan=add", "--enet-vlan-tag=1", "--portmap=53:5353", "--pnat=10.0.0.0/8:192.168.0.0/16",
     "--fixcsum"],
], ids=["tag-pri-cfi", "qinq-seed", "portmap-pnat"])
def test_vlan_add_wave_lane_mixed_shapes(built, args):
    """The wave lane's VLAN push (static +4 placement, tags inserted in the store) on
    v4/v6 TCP/UDP records of odd and even sizes, against the oracle."""
    pcap = _mixed_sizes_pcap(21)
    _, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap)
        assert b.run() == 0
        r = b.result()
        assert r.fast_kind == 2 and r.generic_tiles < r.n_tiles // 2  # the wave lane pushed most tiles
        assert_same(b.output(), exp)
        assert b.run() == 0  # the second run (generic pass left out by the hint) too
        assert_same(b.output(), exp)
        b.close()
    finally:
        te.close()


# ---------------------------------------------------------------- parallel record walk
def test_parallel_walk_survives_fake_record_chains(built, monkeypatch):
    """The host walks a large capture as parallel stretches starting at guessed record
    boundaries.  Payloads full of valid-looking pcap record headers make the guesses
    land inside packets; each wrong guess is caught (the previous stretch does not end
    there) and the walk goes on sequentially, so the output is the oracle's."""
    monkeypatch.setenv("TCPEDIT_HIP_WALK_THREADS", "8")
    fake = b"".join(struct.pack("<IIII", 1, 2, 12, 12) + bytes(range(12)) for _ in range(50))  # 1400 B
    recs = []
    for ts, tu, cl, ln, d in S.records(S.pcap_fixed(8_000, 1_442, seed=31)):
        d = bytearray(d)
        d[42:42 + len(fake)] = fake
        recs.append((ts, tu, cl, ln, bytes(d)))
    pcap = S.build_pcap(recs)
    assert len(pcap) > 10 << 20
    for args in (["--fixcsum"], ["--seed=3", "--fixcsum"]):
        _, exp = O.rewrite(pcap, args)
        rc, out = gpu_rewrite(pcap, args)
        assert rc == 0
        assert_same(out, exp)
        rc, out = pipe_rewrite(pcap, args, chunk=16 << 20)
        assert rc == 0
        assert_same(bytes(out), exp)


def test_parallel_walk_stops_where_libpcap_stops(built, monkeypatch):
    """An oversize record deep in a large capture ends the walk there (libpcap's stop),
    whichever stretch meets it."""
    monkeypatch.setenv("TCPEDIT_HIP_WALK_THREADS", "8")
    recs = S.records(S.pcap_fixed(150_000, 64, seed=32))
    pcap = bytearray(S.build_pcap(recs))
    cut = 24 + 80 * 111_111
    struct.pack_into("<I", pcap, cut + 8, 300_000)  # caplen > 262144: pcap_next stops
    pcap = bytes(pcap)
    _, exp = O.rewrite(pcap, ["--fixcsum"])
    rc, out = gpu_rewrite(pcap, ["--fixcsum"])
    assert_same(out, exp)
    assert len(S.records(out)) == 111_111


# ---------------------------------------------------------------- user / Cisco HDLC encoders
@pytest.mark.parametrize("args,linktype", [
    (["--dlt=user", "--user-dlink=1,2,3,4,5,6,7,8,9,a,b,c,d,e,f,10,11,12,8,0", "--user-dlt=147", "--fixcsum"], 147),
    (["--dlt=user", "--user-dlink=aa,bb,8,0", "--user-dlink=cc,dd,8,0", "--seed=7", "--fixcsum"], 1),
    (["--dlt=hdlc", "--hdlc-address=0x0f", "--hdlc-control=3", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"],
     104),
], ids=["user-20B-longer", "user-client-server", "hdlc"])
def test_dlt_encoders_match_oracle(built, args, linktype):
    """The user and HDLC encoders (L2 header replaced, payload in place, pcap header
    moved; a longer user header into the slot headroom) on v4/v6 TCP/UDP records of
    assorted sizes, VLAN-tagged ones among them, with a tcpprep cache for direction."""
    recs = S.records(_mixed_sizes_pcap(41)) + S.records(G.read("test.pcap"))
    pcap = S.build_pcap(recs)
    cache = S.tcpprep_cache(len(recs), seed=5)
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out = gpu_rewrite(pcap, args, cache)
    assert rc == rc_o
    assert_same(out, exp)
    assert struct.unpack_from("<I", out, 20)[0] == linktype
    te = TA.TcpEdit(args)
    try:
        assert te._L.tcpedit_get_output_dlt(te._ctx) == linktype
    finally:
        te.close()


@pytest.mark.parametrize("n", [40, 200, 255])
def test_dlt_user_header_longer_than_ethernet(built, n):
    """A user header up to USER_L2MAXLEN (255) bytes: the slot headroom is sized from the
    config (te_slot_head), so every length the reference takes is served bit-exact."""
    args = ["--dlt=user", "--user-dlink=" + ",".join(["1"] * n), "--fixcsum"]
    pcap = S.build_pcap(S.records(S.pcap_fixed(100, 64, seed=3)) + S.records(S.pcap_imix(300, seed=4)))
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = gpu_rewrite(pcap, args)
    assert rc == rc_o == 0
    assert_same(out, exp)


# ---------------------------------------------------------------- --fuzz-seed (fuzzing.c)
FUZZ_POOL = [
    ["--fuzz-seed=42", "--fuzz-factor=2"],
    ["--fuzz-seed=7", "--fuzz-factor=1", "--fixcsum"],
    ["--fuzz-seed=1"],
    ["--fuzz-seed=9", "--fuzz-factor=1", "--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"],
    ["--fuzz-seed=3", "--fuzz-factor=1", "--fixlen=pad", "--fixcsum"],
    ["--fuzz-seed=11", "--fuzz-factor=1", "--portmap=1-65535:7", "--tcp-sequence=5", "--ttl=+3", "--tos=9"],
    ["--fuzz-seed=5", "--fuzz-factor=1", "--skip-soft-errors", "--efcs"],
    ["--fuzz-seed=14", "--fuzz-factor=3", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixhdrlen", "--fixcsum"],
    ["--fuzz-seed=12", "--fuzz-factor=1", "--dlt=hdlc", "--hdlc-address=1", "--hdlc-control=2", "--fixcsum"],
    ["--fuzz-seed=13", "--fuzz-factor=1", "--dlt=user", "--user-dlt=147",
     "--user-dlink=1,2,3,4,5,6,7,8,9,a,b,c,d,e,f,10,11,12,8,0", "--fixcsum"],
    ["--fuzz-seed=0", "--fuzz-factor=1", "--mtu-trunc", "--mtu=200", "--fixcsum"],
    ["--fuzz-seed=21", "--fuzz-factor=1", "--enet-vlan=del", "--tclass=3", "--flowlabel=77"],
]


@pytest.mark.parametrize("k", range(len(FUZZ_POOL)))
def test_fuzz_matches_oracle_on_mixed_captures(built, k):
    """One RNG draw per record that reaches the fuzz step, in record order, over many
    tiles and scan blocks (reach pass + prefix count + LCG jump), then the reference's
    second L2/L3 pass; v4/v6 TCP/UDP of assorted sizes, the golden capture, a cache."""
    args = FUZZ_POOL[k]
    gold = S.records(G.read("test.pcap"))
    recs = S.records(_mixed_sizes_pcap(60 + k)) + (mutate(gold, random.Random(k)) if k % 2 else gold)
    pcap = S.build_pcap(recs)
    cache = S.tcpprep_cache(len(recs), seed=k, nosend_every=13) if k % 3 == 0 else None
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out, st = gpu_rewrite(pcap, args, cache, with_status=True)
    assert not (st & TA.ST.UNSUPPORTED).any()  # stale-buffer reads (Q8) are replayed
    assert rc == rc_o
    assert_same(out, exp)


def test_fuzz_state_runs_across_a_million_records(built):
    """> 1024 x 1024 records: the block-count scan loops, and ranks reach 2^20."""
    pcap = S.pcap_fixed(1_100_000, 60, seed=31)
    args = ["--fuzz-seed=77", "--fuzz-factor=3", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = gpu_rewrite(pcap, args)
    assert rc == rc_o == 0
    assert_same(out, exp)


def test_fuzz_state_carries_across_pipelined_chunks_and_runs(built):
    """The context's RNG state carries from chunk to chunk (fuzzing_init runs once per
    context), so a chunked run equals one oracle run; a second run continues the stream."""
    pcap = S.pcap_imix(30_000, seed=32)
    args = ["--fuzz-seed=99", "--fuzz-factor=2", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    rc, out = pipe_rewrite(pcap, args, chunk=1 << 20)
    assert rc == rc_o == 0
    assert_same(out, exp)
    # two batches through one context == one oracle run over their concatenation
    recs = S.records(pcap)
    a, b = S.build_pcap(recs[:12_345]), S.build_pcap(recs[12_345:])
    te = TA.TcpEdit(args)
    try:
        rc1, out1 = te.rewrite(a)
        rc2, out2 = te.rewrite(b)
    finally:
        te.close()
    assert rc1 == rc2 == 0
    assert S.records(out1) + S.records(out2) == S.records(exp)


def test_fuzz_through_the_per_packet_api(built):
    recs = S.records(G.read("test.pcap"))
    args = ["--fuzz-seed=42", "--fuzz-factor=2"]
    _, exp = O.rewrite(S.build_pcap(recs), args)
    te = TA.TcpEdit(args)
    got = []
    try:
        for ts, tu, cl, ln, data in recs:
            buf = bytearray(262166)
            buf[:cl] = data
            rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf)
            assert rc != TA.TCPEDIT_ERROR
            if h["caplen"]:
                got.append((ts, tu, h["caplen"], h["len"], bytes(buf[:h["caplen"]])))
    finally:
        te.close()
    assert got == S.records(exp) == S.records(G.read("test2.rewrite_l7fuzzing"))
