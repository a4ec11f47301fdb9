"""safe_pcap_next's rules in the oracle (CPU): the record read every caller of the edit makes
-- tcprewrite.c:289, tcpprep.c:353, send_packets.c:955,985 -> src/common/utils.c:131-169:

  * len > MAX_SNAPLEN, len == 0 or caplen == 0: an error message and exit(-1) (:136-156); the
    output keeps the records written before (tcprewrite's and tcpreplay's pcap_dump), and
    tcpprep writes no cache (write_cache comes after the pass, tcpprep.c:194);
  * len < caplen: caplen = len before the copy and the edit (:159-162); the reader moves on
    past the record as stored.

Parity unpinned: no reference fixture holds such a record (test.pcap has caplen == len
throughout).  The expected results here are built from the reference's own goldens and
from the same capture with the record pre-trimmed, independently of the oracle's reader.
The GPU is checked against the oracle on these records in test_gpu_parity.py (mutated
captures), test_device_index.py, test_fused.py and test_tcpprep_gpu.py."""
import struct

import pytest

import golden_cases as G
import oracle_lib as O
import tcpprep_cases as T
from tcpreplay_amd import synth as S


def _with(recs, k, rec):
    r = list(recs)
    r[k] = rec
    return S.build_pcap(r)


@pytest.mark.parametrize("zc,zl", [(0, 0), (0, 60), (60, 0), (60, 262145)])
@pytest.mark.parametrize("case", ["test2.rewrite_fixcsum", "test2.rewrite_seed", "test2.rewrite_pnat",
                                  "test2.rewrite_config", "test2.rewrite_efcs"])
def test_tcprewrite_stops_before_the_record(built, zc, zl, case):
    """the output is the golden's first k records, and the run fails (rc -1)"""
    name, inp, cache, args, _ = next(c for c in G.IN_SCOPE if c[0] == case)
    recs = S.records(G.read(inp))
    k = 77
    ts, tu, cl, ln, d = recs[k]
    pcap = _with(recs, k, (ts, tu, zc, zl, d[:zc]))
    rc, out = O.rewrite(pcap, args, G.read(cache) if cache else None)
    gold = G.read(name)
    assert rc == -1
    assert out[:24] == gold[:24]
    assert S.records(out) == S.records(gold)[:k]


@pytest.mark.parametrize("args", [["--fixcsum"], ["--seed=42", "--fixcsum"], ["--efcs"],
                                  ["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"],
                                  ["--mtu-trunc", "--mtu=100", "--fixcsum"], ["--ttl=9"]])
def test_tcprewrite_trims_caplen_to_len(built, args):
    """a len < caplen record edits and writes as the same record stored with caplen = len
    (its bytes past len never read): padded frames, a cut inside L4, one byte left"""
    recs = S.records(G.read("test.pcap"))
    stored, trimmed = list(recs), list(recs)
    for k, keep in ((14, 42), (15, 34), (20, 30), (30, 1), (40, 14), (50, 20)):
        ts, tu, cl, ln, d = recs[k]
        junk = bytes((b ^ 0x5a) for b in d[keep:])  # bytes the reader must not pass on
        stored[k] = (ts, tu, cl, keep, d[:keep] + junk)
        trimmed[k] = (ts, tu, keep, keep, d[:keep])
    rc1, out1 = O.rewrite(S.build_pcap(stored), args)
    rc2, out2 = O.rewrite(S.build_pcap(trimmed), args)
    assert rc1 == rc2 == 0
    assert out1 == out2


def test_trim_moves_the_stale_buffer_extent(built):
    """the copy is the trimmed caplen (tcprewrite.c:301): a later record reading past its own
    bytes sees what the trimmed copy left, not the stored record's tail"""
    ts, tu, cl, ln, d = S.records(S.pcap_fixed(1, 200, ipv6=True, proto=17, seed=3))[0]
    d = bytearray(d)
    struct.pack_into(">H", d, 18, struct.unpack_from(">H", d, 18)[0] + 50)  # payload length +50
    big = (ts, tu, 1200, 1200, bytes(range(256)) * 4 + bytes(176))
    tail = big[4][:150] + b"\xee" * 1050  # a stored tail the copy must leave out
    stored = [big, (ts, tu, 1200, 150, tail), (ts, tu, cl, ln, bytes(d))]
    trimmed = [big, (ts, tu, 150, 150, big[4][:150]), (ts, tu, cl, ln, bytes(d))]
    whole = [big, (ts, tu, 1200, 1200, tail), (ts, tu, cl, ln, bytes(d))]
    a = O.rewrite(S.build_pcap(stored), ["--fixcsum"])
    b = O.rewrite(S.build_pcap(trimmed), ["--fixcsum"])
    c = O.rewrite(S.build_pcap(whole), ["--fixcsum"])
    assert a == b
    assert S.records(a[1])[2] != S.records(c[1])[2]  # (the stale bytes do reach the checksum)


@pytest.mark.parametrize("zc,zl", [(0, 0), (0, 60), (60, 0), (60, 300_000)])
def test_tcpprep_writes_no_cache(built, zc, zl):
    recs = S.records(T.test_pcap())
    ts, tu, cl, ln, d = recs[100]
    pcap = _with(recs, 100, (ts, tu, zc, zl, d[:zc]))
    for args in (["--port"], ["--auto=bridge"], ["--mac=00:1f:f3:3c:e1:13"]):
        with pytest.raises(ValueError, match="-5"):
            O.tcpprep(pcap, args)


def test_tcpprep_trims_caplen_to_len(built):
    """len < caplen classifies as the record stored with caplen = len (a short IPv4 header
    is non-IP; MAC mode gives a record trimmed below 14 bytes no entry)"""
    recs = S.records(T.test_pcap())
    stored, trimmed = list(recs), list(recs)
    for k, keep in ((3, 10), (9, 30), (19, 40), (40, 13), (60, 1)):
        ts, tu, cl, ln, d = recs[k]
        stored[k] = (ts, tu, cl, keep, d)
        trimmed[k] = (ts, tu, keep, keep, d[:keep])
    def run(pcap, args):
        try:
            return O.tcpprep(pcap, args)
        except ValueError as e:  # (auto modes: packet2tree's abort on a trimmed short TCP record)
            return str(e)
    for name in sorted(T.CASES):
        args = T.args(name)
        assert run(S.build_pcap(stored), args) == run(S.build_pcap(trimmed), args), name


def test_tcpreplay_edit_stops_after_the_records_before(built):
    """tcpreplay-edit -w: the first pass sends the records before the bad one, then exits
    (the later --loop passes never run)"""
    recs = S.records(G.read("test.pcap"))
    ts, tu, cl, ln, d = recs[90]
    pcap = _with(recs, 90, (ts, tu, cl, 0, d))
    rc, dump = O.replay_edit(pcap, ["--fixcsum"], loops=3)
    rc1, one = O.replay_edit(S.build_pcap(recs[:90]), ["--fixcsum"], loops=1)
    assert rc == -1 and rc1 == 0
    assert dump == one


def test_tcpreplay_edit_trims_caplen_to_len(built):
    recs = S.records(G.read("test.pcap"))
    stored, trimmed = list(recs), list(recs)
    for k, keep in ((14, 42), (33, 20)):
        ts, tu, cl, ln, d = recs[k]
        stored[k] = (ts, tu, cl, keep, d)
        trimmed[k] = (ts, tu, keep, keep, d[:keep])
    for preload in (False, True):
        a = O.replay_edit(S.build_pcap(stored), ["--enet-vlan=add", "--enet-vlan-tag=9"], loops=3, preload=preload)
        b = O.replay_edit(S.build_pcap(trimmed), ["--enet-vlan=add", "--enet-vlan-tag=9"], loops=3, preload=preload)
        assert a == b


def test_tcpreplay_unique_ip_reader_rules(built):
    """tcpreplay -w --unique-ip: the exit keeps the first pass's earlier records; a trimmed
    record is sent as len bytes"""
    import ctypes
    lib = O.load()
    lib.tcpreplay_oracle_exited.restype = ctypes.c_int
    recs = S.records(G.read("test.pcap"))
    ts, tu, cl, ln, d = recs[120]
    bad = _with(recs, 120, (ts, tu, 0, ln, b""))
    out, _ = O.replay(bad, ["--unique-ip", "--loop=2"])
    assert lib.tcpreplay_oracle_exited() == 1
    ref, _ = O.replay(S.build_pcap(recs[:120]), ["--unique-ip", "--loop=1"])
    assert lib.tcpreplay_oracle_exited() == 0
    assert out == ref
    stored, trimmed = list(recs), list(recs)
    stored[7] = (ts, tu, cl, 40, d)
    trimmed[7] = (ts, tu, 40, 40, d[:40])
    assert O.replay(S.build_pcap(stored), ["--unique-ip", "--loop=3"]) == \
        O.replay(S.build_pcap(trimmed), ["--unique-ip", "--loop=3"])
