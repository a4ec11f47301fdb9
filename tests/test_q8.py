"""edits that read the reference's stale static packet buffer.

tcprewrite memcpy's every record into one never-cleared MAXPACKET buffer
(tcprewrite.c:267-301); an IPv6 checksum over an overstated payload length, a TCP
sequence field or ARP address past caplen, or remap_ipv6's stray write reads what
earlier records (as edited) left there.  The device lists such records and replays the
buffer (te_q8_replay); the oracle keeps the reference's static buffer itself.  Every
case here must come out byte-identical to the oracle -- or, where the bytes come from
outside the batch (a later pipeline chunk), fail loudly.
"""
import random
import struct

import pytest

import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu


def _overstate(recs, idxs, by=50):
    """IPv6 records whose payload length claims `by` more bytes than were captured"""
    recs = list(recs)
    for i in idxs:
        ts, tu, cl, ln, d = recs[i]
        d = bytearray(d)
        assert d[12:14] == b"\x86\xdd"
        struct.pack_into(">H", d, 18, struct.unpack_from(">H", d, 18)[0] + by)
        recs[i] = (ts, tu, cl, ln, bytes(d))
    return recs


def _mixed(n, seed):
    rng = random.Random(seed)
    parts = []
    for size, v6, proto in [(90, True, 17), (97, True, 6), (200, True, 17), (333, False, 6), (1514, True, 17),
                            (64, False, 17), (600, True, 6)]:
        parts += S.records(S.pcap_fixed(n, size, seed=rng.randrange(1 << 20), ipv6=v6, proto=proto))
    rng.shuffle(parts)
    return parts


def _gpu(pcap, args, cache=None):
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap, cache)
        rc = b.run()
        out, r = b.output(), b.result()
        b.close()
        return rc, out, r
    finally:
        te.close()


def _check(pcap, args, cache=None, min_stale=1):
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out, r = _gpu(pcap, args, cache)
    assert r.stale_records >= min_stale, "the case must exercise the replay"
    assert r.unsupported == 0
    assert rc == rc_o
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"


@pytest.mark.parametrize("args", [["--fixcsum"], ["--seed=9", "--fixcsum"], ["--enet-vlan=add", "--enet-vlan-tag=5",
                                  "--fixcsum"], ["--efcs", "--fixcsum"], ["--fixlen=pad", "--fixcsum"],
                                  ["--pnat=[::/0]:[2001:db8:aaaa::/36]", "--fixcsum"]])
def test_overstated_ipv6_payloads_read_earlier_records(built, args):
    """IPv6 records with overstated payload lengths amid records of other sizes: the
    checksum sums bytes the previous records (as edited) left in the buffer"""
    recs = _mixed(60, seed=len(args))
    v6 = [i for i, r in enumerate(recs) if r[4][12:14] == b"\x86\xdd" and r[2] >= 90]
    pick = sorted(random.Random(7).sample(v6, 25))
    _check(S.build_pcap(_overstate(recs, pick)), args, min_stale=5)


def test_stale_bytes_from_the_capture_start_are_zeros(built):
    """the first record reads past its caplen: the reference's buffer starts zeroed"""
    recs = S.records(S.pcap_fixed(5, 200, ipv6=True, proto=17, seed=3))
    _check(S.build_pcap(_overstate(recs, [0, 1, 2, 3, 4])), ["--fixcsum"], min_stale=5)


def test_vlan_delete_leaves_the_old_tail(built):
    """VLAN-tagged records shrink by 4 (--enet-vlan=del): the reference's buffer keeps
    the old last 4 bytes past the new end, where the next record's overread lands"""
    base = S.records(S.pcap_fixed(40, 300, ipv6=True, proto=17, seed=5))
    recs = []
    for k, (ts, tu, cl, ln, d) in enumerate(base):
        if k % 2 == 0:  # tagged, longer: its tail covers the next record's overread
            d = d[:12] + b"\x81\x00\x00\x07" + d[12:] + bytes(range(40))
            cl = ln = len(d)
        recs.append((ts, tu, cl, ln, d))
    recs = _overstate(recs, [k for k in range(1, 40, 2)], by=30)
    _check(S.build_pcap(recs), ["--enet-vlan=del", "--fixcsum"], min_stale=10)


def test_truncated_tcp_header_sequence_edit(built):
    """--tcp-sequence on a TCP header cut by the capture reads and rewrites fields past
    caplen: nothing of that reaches its own output, but it is in the buffer"""
    big = S.records(S.pcap_fixed(4, 400, ipv6=False, proto=6, seed=8))
    v6 = S.records(S.pcap_fixed(4, 200, ipv6=True, proto=6, seed=9))
    recs = []
    for k in range(4):
        ts, tu, cl, ln, d = big[k]
        recs.append((ts, tu, cl, ln, d))
        ts, tu, cl, ln, d = big[(k + 1) % 4]
        recs.append((ts, tu, 40, ln, d[:40]))  # TCP header cut after 6 bytes: seq fields are stale
        recs.append(_overstate([v6[k]], [0], by=150)[0])
    _check(S.build_pcap(recs), ["--tcp-sequence=77", "--fixcsum"], min_stale=4)


@pytest.mark.parametrize("seed", range(6))
def test_mutated_captures_with_stale_reads(built, seed):
    """random header mutations (truncations, len != caplen, tags) over a v4/v6 mix with
    overstated IPv6 payloads: every option line of the differential pool"""
    import test_gpu_parity as P
    rng = random.Random(100 + seed)
    recs = P.mutate(_mixed(25, seed=seed), rng)
    v6 = [i for i, r in enumerate(recs) if r[4][12:14] == b"\x86\xdd" and r[2] >= 60]
    recs = _overstate(recs, rng.sample(v6, min(12, len(v6))), by=rng.randrange(1, 300))
    pcap = S.build_pcap(recs)
    for args in P.OPTION_POOL[seed::6]:
        rc_o, exp = O.rewrite(pcap, args)
        rc, out, r = _gpu(pcap, args)
        assert r.unsupported == 0 and rc == rc_o and out == exp, args


def test_pipelined_chunks_replay_across_chunk_boundaries(built):
    """chunk 0 starts at the capture's start; a later chunk's replay walks back into the
    earlier chunks' records (tcprewrite's buffer carries across the whole run,
    tcprewrite.c:267-280): a donor just before the chunk, and one that is the capture's
    zeroed start two chunks back"""
    recs = S.records(S.pcap_fixed(30_000, 90, ipv6=True, proto=17, seed=11))
    cover = S.records(S.pcap_fixed(1, 400, ipv6=True, proto=17, seed=12))[0]
    recs[20_001] = cover  # a longer record just before the overread covers it
    te = TA.TcpEdit(["--fixcsum"])
    try:
        for bad in ([3, 20_002], [9_600, 10_400], [15_000], [25_000]):
            pcap = S.build_pcap(_overstate(recs, bad, by=40))
            rc_o, exp = O.rewrite(pcap, ["--fixcsum"])
            rc, out = te.rewrite_pipelined(pcap, chunk_bytes=1 << 20)
            assert rc == rc_o == 0, (bad, te.geterr())
            assert out == exp, bad
    finally:
        te.close()


def test_pipelined_replay_prefix_starts_at_a_chunk_anchor(built):
    """past the first ~33 MiB a chunk's replay prefix walk starts at an earlier chunk's first
    record (bounded work per retry): the donors of stale bytes a few thousand
    records back are staged from there"""
    n = 420_000  # 90-byte records: ~44 MiB
    recs = S.records(S.pcap_fixed(n, 90, ipv6=True, proto=17, seed=21))
    cover = S.records(S.pcap_fixed(1, 400, ipv6=True, proto=17, seed=22))[0]
    recs[399_990] = recs[409_000] = cover  # longer records a little before the overreads cover them
    recs = _overstate(recs, [400_001, 410_000, 412_000], by=40)
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, ["--fixcsum"])
    te = TA.TcpEdit(["--fixcsum"])
    try:
        rc, out = te.rewrite_pipelined(pcap, chunk_bytes=8 << 20)
        assert rc == rc_o == 0, te.geterr()
        assert out == exp
    finally:
        te.close()


def test_batch_prefix_records_feed_the_replay(built):
    """a batch that starts mid-capture (a shard) with the records before it staged as its
    prefix equals the oracle's whole-capture output over its records; without the prefix the
    record is refused loudly"""
    recs = S.records(S.pcap_fixed(4_000, 90, ipv6=True, proto=17, seed=13))
    recs[1_990] = S.records(S.pcap_fixed(1, 500, ipv6=True, proto=17, seed=14))[0]
    recs = _overstate(recs, [2_005, 3_100], by=60)
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, ["--fixcsum"])
    cut = 24 + sum(16 + r[2] for r in recs[:2_000])
    exp_tail = exp[24 + sum(16 + r[2] for r in S.records(exp)[:2_000]):]
    for with_prefix in (True, False):
        te = TA.TcpEdit(["--fixcsum"])
        try:
            b = TA.Batch(te, memoryview(pcap)[cut:], pkt_base=2_000, hdr=pcap[:24])
            if with_prefix:
                b.set_prefix(memoryview(pcap)[24:cut])
            rc = b.run()
            if with_prefix:
                assert rc == 0, te.geterr()
                r = b.result()
                got = bytearray(r.out_len - 24)
                assert b.output_records_into(got) == len(got)
                assert r.stale_records >= 2 and r.unsupported == 0
                assert bytes(got) == exp_tail
            else:
                assert rc == TA.TCPEDIT_ERROR and "stale static packet buffer" in te.geterr()
            b.close()
        finally:
            te.close()


def test_per_packet_api_reads_the_callers_buffer(built):
    """tcpedit_packet edits the caller's buffer: with one buffer reused for every record
    (tcprewrite's rewrite_packets) the stale bytes are the previous records', as the
    oracle's static buffer has them"""
    recs = _mixed(8, seed=3)
    v6 = [i for i, r in enumerate(recs) if r[4][12:14] == b"\x86\xdd" and r[2] >= 90]
    recs = _overstate(recs, v6[::3])
    pcap = S.build_pcap(recs)
    _, exp = O.rewrite(pcap, ["--fixcsum"])
    te = TA.TcpEdit(["--fixcsum"])
    buf = bytearray(262166)
    got = []
    try:
        for ts, tu, cl, ln, d in recs:
            buf[:cl] = d
            rc, h = te.packet({"ts_sec": ts, "ts_usec": tu, "caplen": cl, "len": ln}, buf)
            assert rc != TA.TCPEDIT_ERROR, te.geterr()
            got.append((ts, tu, h["caplen"], h["len"], bytes(buf[:h["caplen"]])))
    finally:
        te.close()
    assert got == S.records(exp)


def test_trimmed_records_bound_the_stale_extent(built):
    """a len < caplen record is copied as len bytes (safe_pcap_next's trim, utils.c:159-162,
    then tcprewrite.c:301): the stale bytes a later overstated IPv6 record reads are the
    older record's past that, not the trimmed record's stored tail"""
    ts, tu, cl, ln, d = S.records(S.pcap_fixed(1, 200, ipv6=True, proto=17, seed=3))[0]
    v6 = _overstate([(ts, tu, cl, ln, d)], [0])[0]
    big = S.records(S.pcap_fixed(1, 1200, seed=4))[0]
    recs = []
    for k in range(40):
        keep = 120 + 7 * k
        tail = big[4][:keep] + bytes([0xE0 + (k & 15)]) * (1200 - keep)
        recs += [big, (ts, tu, 1200, keep, tail), v6]
    _check(S.build_pcap(recs), ["--fixcsum"], min_stale=40)
