"""tcpreplay --unique-ip (src/send_packets.c:124-257, :362-372, :477-483) and the
--include / --exclude packet list (:440-447, src/common/list.c) with file output (-w):
the reference's goldens test2.replay_unique_ip, test2.replay_include and
test2.replay_exclude (test/Makefile.am:214-216, `tcpreplay -w ... -t <opts> test.pcap`),
the oracle (oracle/tcpreplay_oracle.c) pinned to them, and the device passes
(tcpreplay_kernels.hip) against both, bit-exact."""
import random
import struct

import pytest

import golden_cases as G
import oracle_lib as O
from tcpreplay_amd import synth as S

GOLDEN_ARGS = ["--unique-ip", "--loop=2"]


def _golden():
    return G.read("test2.replay_unique_ip")


def test_oracle_reproduces_the_reference_golden(built):
    out, failed = O.replay(G.read("test.pcap"), GOLDEN_ARGS)
    assert out == _golden()
    assert failed == 3  # the non-IP records of pass 2 (ARP, 802.3) are counted and not sent


def test_oracle_pass_structure(built):
    """pass 1 is the capture as read (timestamp fractions x1000, the nanosecond read);
    --loop=1 edits nothing; -K edits the cached records cumulatively"""
    pcap = G.read("test.pcap")
    one, f1 = O.replay(pcap, ["--unique-ip"])
    assert f1 == 0 and len(S.records(one)) == len(S.records(pcap))
    r_in, r_out = S.records(pcap), S.records(one)
    assert all(a[4] == b[4] and b[1] == (a[1] * 1000) & 0xFFFFFFFF for a, b in zip(r_in, r_out))
    cached, fc = O.replay(pcap, ["--unique-ip", "--loop=3", "-K"])
    plain, fp = O.replay(pcap, ["--unique-ip", "--loop=3"])
    assert fc == fp == 6 and len(S.records(cached)) == len(S.records(plain)) == 3 * 179 - 6
    # the third pass shifts each address by 2 from the capture's (uncached: by the iteration;
    # cached: one more step on the cached record) -- the wrap edges differ (test_gpu_*_wrap_edges)
    third = 179 + 176  # pass 1 sends every record, the edit passes all but the 3 non-IP ones
    assert [r[4] for r in S.records(cached)[third:]] == [r[4] for r in S.records(plain)[third:]]


def _edge_pcap(n=2000, seed=3):
    """IPv4 / IPv6 (src/dst word 3) near the wrap points, equal addresses, VLAN tags,
    non-IP and too-short records"""
    rng = random.Random(seed)
    v4 = S.records(S.pcap_fixed(n, 64, seed=seed))
    v6 = S.records(S.pcap_fixed(n // 2, 90, ipv6=True, seed=seed + 1))
    picks = [0, 1, 2, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF]
    recs = []
    for i, (ts, tu, cl, ln, d) in enumerate(v4 + v6):
        d = bytearray(d)
        v6r = d[12:14] == b"\x86\xdd"
        s_at, d_at = (34, 50) if v6r else (26, 30)
        for at in (s_at, d_at):
            x = rng.choice(picks) if rng.random() < 0.5 else rng.randrange(1 << 32)
            d[at:at + 4] = struct.pack(">I", x)
        if i % 17 == 0:
            d[d_at:d_at + 4] = d[s_at:s_at + 4]
        if i % 23 == 0:
            d = d[:12] + b"\x81\x00\x00\x05" + d[12:]
        if i % 29 == 0:
            d[12:14] = b"\x08\x06"  # ARP: not sent on an edit pass
        if i % 31 == 0:
            d = d[:20]  # too short for an IP header
        recs.append((ts, tu, len(d), len(d), bytes(d)))
    rng.shuffle(recs)
    return S.build_pcap(recs)


@pytest.mark.gpu
def test_gpu_reproduces_the_reference_golden(built):
    from tcpreplay_amd import tcpreplay as TR
    out, failed = TR.replay(G.read("test.pcap"), GOLDEN_ARGS)
    assert out == _golden() and failed == 3


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ["--unique-ip", "--loop=4"],
    ["--unique-ip", "--loop=5", "--unique-ip-loops=2"],
    ["--unique-ip", "--loop=4", "-K"],
    ["--unique-ip", "--loop=6", "--unique-ip-loops=3", "--preload-pcap"],
    ["--loop=2"],
], ids=["loop4", "uloops2", "preload", "preload-uloops3", "no-unique"])
def test_gpu_matches_oracle_on_wrap_edges(built, args):
    from tcpreplay_amd import tcpreplay as TR
    pcap = _edge_pcap()
    assert TR.replay(pcap, args) == O.replay(pcap, args)


@pytest.mark.gpu
def test_gpu_nanosecond_and_big_endian_input(built):
    """a nanosecond capture keeps its fraction; a big-endian one is written little-endian"""
    from tcpreplay_amd import tcpreplay as TR
    recs = S.records(_edge_pcap(300, seed=9))
    for magic in (0xA1B23C4D, 0xD4C3B2A1):
        sw = magic == 0xD4C3B2A1
        e = ">" if sw else "<"
        hdr = struct.pack(e + "IHHiIII", 0xA1B2C3D4 if sw else magic, 2, 4, 0, 0, 65535, 1)
        body = b"".join(struct.pack(e + "IIII", ts, tu, cl, ln) + d for ts, tu, cl, ln, d in recs)
        pcap = hdr + body
        assert TR.replay(pcap, ["--unique-ip", "--loop=3"]) == O.replay(pcap, ["--unique-ip", "--loop=3"])


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--unique-ip", "--loop=4"], ["--unique-ip", "--loop=3", "-K"], ["--loop=2"]],
                         ids=["loop4", "preload", "no-unique"])
def test_gpu_reader_rules_match_oracle(built, args):
    """safe_pcap_next's rules (send_packets.c:955,985 -> src/common/utils.c:131-169): len <
    caplen records are sent as len bytes; a zero len or caplen record ends the run after the
    first pass's earlier records (TCPREPLAY_HIP_READER_EXIT: ReaderExit carries that output,
    geterr names the record)"""
    import ctypes
    from tcpreplay_amd import tcpreplay as TR
    lib = O.load()
    lib.tcpreplay_oracle_exited.restype = ctypes.c_int
    recs = S.records(_edge_pcap(400, seed=11))
    for i in range(3, len(recs), 37):
        ts, tu, cl, ln, d = recs[i]
        recs[i] = (ts, tu, cl, max(1, cl - 1 - i % 30), d)
    pcap = S.build_pcap(recs)
    t = TR.TcpReplay(args)
    try:
        assert t.replay(pcap) == O.replay(pcap, args)
        assert not t.reader_exited and lib.tcpreplay_oracle_exited() == 0
        for zc, zl in ((0, 0), (0, 70), (70, 0)):
            ts, tu, cl, ln, d = recs[250]
            bad = S.build_pcap(recs[:250] + [(ts, tu, zc, zl, d[:zc])] + recs[251:])
            with pytest.raises(TR.ReaderExit) as ex:
                t.replay(bad)
            assert t.reader_exited and "safe_pcap_next" in str(ex.value)
            assert (ex.value.output, ex.value.failed) == O.replay(bad, args) and lib.tcpreplay_oracle_exited() == 1
    finally:
        t.close()


def test_unserved_options_are_refused(built):
    from tcpreplay_amd import tcpreplay as TR
    for bad in (["--unique-ip-loops=2"], ["--loop=0"], ["--mbps=10"], ["--unique-ip", "--unique-ip-loops=0"]):
        with pytest.raises(ValueError):
            TR.TcpReplay(bad)


# ------------------------------------------------------ --include / --exclude (list.c)
LIST_GOLDENS = [("test2.replay_include", ["--include=7,11,20-23,174-"]),
                ("test2.replay_exclude", ["--exclude=23-,11-20,2,3"])]
LIST_LINES = [
    ["--include=1-100,500-"], ["--exclude=0-50"], ["--include=010,2-"],  # 010: strtoull base 0 (octal 8)
    ["--exclude=3- "], ["--include=5,5,5,0"], ["--include=2000-1500"],  # an empty range
    ["--include=1-300,700-900", "--unique-ip", "--loop=3"],
    ["--exclude=2-20,40-", "--unique-ip", "--loop=3", "-K"],
    ["--include=3-", "--unique-ip", "--unique-ip-loops=2", "--loop=5"],
]


@pytest.mark.parametrize("name,args", LIST_GOLDENS)
def test_oracle_reproduces_the_list_goldens(built, name, args):
    out, failed = O.replay(G.read("test.pcap"), args)
    assert out == G.read(name) and failed == 0


def test_unparsable_lists_are_refused(built):
    """parse_list's regex (list.c:72) refuses the whole list; --include and --exclude
    exclude each other (tcpreplay_opts.def:310,340)"""
    from tcpreplay_amd import tcpreplay as TR
    for bad in (["--include=a"], ["--include=5-x"], ["--include=,"], ["--exclude=-3"], ["--include=1", "--exclude=2"],
                ["--include=1 "]):
        with pytest.raises(ValueError):
            TR.TcpReplay(bad)


@pytest.mark.gpu
@pytest.mark.parametrize("name,args", LIST_GOLDENS)
def test_gpu_reproduces_the_list_goldens(built, name, args):
    from tcpreplay_amd import tcpreplay as TR
    out, failed = TR.replay(G.read("test.pcap"), args)
    assert out == G.read(name) and failed == 0


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(LIST_LINES)))
def test_gpu_lists_match_the_oracle(built, k):
    """the list with --unique-ip, --loop and -K: a listed-out record is neither edited (the
    -K cache keeps it) nor sent nor counted failed"""
    from tcpreplay_amd import tcpreplay as TR
    args = LIST_LINES[k]
    for pcap in (G.read("test.pcap"), _edge_pcap(1500, seed=k + 9)):
        exp = O.replay(pcap, args)
        assert TR.replay(pcap, args) == exp
