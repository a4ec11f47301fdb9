"""The register-resident fast lane (fast_lane.hpp + te_fast_tiles) against the
oracle, bit-exact, and against the generic lane (TCPEDIT_HIP_NO_FAST=1)."""
import os
import struct

import pytest

import fl_cases as F
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu

FAST_OPTION_SETS = [
    ["--fixcsum"],
    ["--seed=42", "--fixcsum"],
    ["--seed=7", "--skipbroadcast", "--fixcsum"],
    ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"],
    ["--portmap=1-65535:7", "--fixcsum"],
    ["--srcipmap=0.0.0.0/0:10.1.0.0/16", "--dstipmap=172.0.0.0/8:11.0.0.0/8", "--fixcsum"],
    ["--pnat=[2001::/16]:[2001:db8:aaaa::/48],[2606::/16]:[fd00::/8]", "--fixcsum"],
    ["--enet-dmac=00:12:13:14:15:16", "--enet-smac=00:22:33:44:55:66", "--fixcsum"],
    ["--enet-dmac=00:12:13:14:15:16", "--enet-smac=00:22:33:44:55:66", "--skipl2broadcast", "--fixcsum"],
    ["--seed=99", "--portmap=443:8443", "--pnat=172.16.0.0/12:10.99.0.0/16", "--fixcsum"],
    # --enet-subsmac (applied in list order, each entry on the earlier ones' result) and
    # --enet-mac-seed (per-byte masks past the kept bytes, unicast addresses only) on the
    # wave lane (en10mb.c:659-689)
    ["--enet-subsmac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee", "--enet-subsmac=00:aa:bb:cc:dd:ee,01:00:5e:00:00:07",
     "--enet-subsmac=00:66:77:88:99:aa,ff:ff:ff:ff:ff:ff", "--fixcsum"],
    ["--enet-mac-seed=42", "--fixcsum"],
    ["--enet-mac-seed=7", "--enet-mac-seed-keep-bytes=3", "--seed=5", "--fixcsum"],
    ["--enet-mac-seed=9", "--enet-mac-seed-keep-bytes=1", "--ttl=+2"],
    ["--enet-subsmac=00:11:22:33:44:55,00:12:34:56:78:9a", "--enet-dmac=00:12:13:14:15:16", "--skipl2broadcast",
     "--fixcsum"],
]


def run(pcap, args, cache=None):
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap, cache)
    try:
        rc = b.run()
        return rc, b.output(), b.result()
    finally:
        b.close()
        te.close()


def first_diff(a, b):
    n = min(len(a), len(b))
    return next((i for i in range(n) if a[i] != b[i]), n)


@pytest.mark.parametrize("k", range(len(FAST_OPTION_SETS)))
def test_fast_lane_mixed_shapes_match_oracle(built, k):
    args = FAST_OPTION_SETS[k]
    pcap = F.build(F.mixed(6000, seed=100 + k))
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, r = run(pcap, args)
    assert r.fast_lane == 1
    assert rc == rc_o
    assert out == exp, f"first difference at byte {first_diff(out, exp)}"


@pytest.mark.parametrize("k", [0, 1, 3, 6])
def test_fast_lane_pure_fast_shapes_never_defer(built, k):
    args = FAST_OPTION_SETS[k]
    pcap = F.build(F.mixed(3000, seed=7 + k, near_miss=0.0))
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, r = run(pcap, args)
    assert r.fast_lane == 1 and r.generic_tiles == 0
    assert rc == rc_o == 0 and out == exp


@pytest.mark.parametrize("args", [["--seed=42", "--fixcsum"],
                                  ["--portmap=53:5353", "--seed=5", "--fixcsum"],
                                  ["--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"]])
def test_udp_checksum_that_updates_to_zero_is_kept(built, args):
    """Every value of the UDP checksum field on the same datagram: for each update
    chain exactly one value comes out of the incremental updates as 0, and then
    --fixcsum leaves it 0 (checksum.c:115)."""
    base = S.records(S.pcap_fixed(1, 64, seed=3))[0]
    ts, tu, cl, ln, d = base
    d = bytearray(d)
    d[36:38] = struct.pack("!H", 53)  # a mapped port
    recs = []
    for v in range(65536):
        e = bytearray(d)
        e[40:42] = struct.pack("<H", v)
        recs.append((ts, tu, cl, ln, bytes(e)))
    pcap = S.build_pcap(recs)
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, r = run(pcap, args)
    assert r.fast_lane == 1 and r.generic_tiles == 0
    assert rc == rc_o == 0 and out == exp
    outs = S.records(out)
    assert any(rec[4][40:42] == b"\0\0" for rec in outs[1:])  # the zero case is really hit


def test_fast_and_generic_lanes_agree(built):
    pcap = F.build(F.mixed(8000, seed=55))
    args = ["--seed=11", "--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=80:8080", "--fixcsum"]
    rc1, out1, r1 = run(pcap, args)
    os.environ["TCPEDIT_HIP_NO_FAST"] = "1"
    try:
        rc2, out2, r2 = run(pcap, args)
    finally:
        del os.environ["TCPEDIT_HIP_NO_FAST"]
    assert r1.fast_lane == 1 and r2.fast_lane == 0
    assert rc1 == rc2 and out1 == out2


def test_fast_lane_huge_and_jumbo_records(built):
    rng_recs = F.mixed(200, seed=5, near_miss=0.0)
    big = (S.records(S.pcap_fixed(2, 9000, seed=2)) + S.records(S.pcap_fixed(1, 20000, seed=3, ipv6=True, proto=6))
           + S.records(S.pcap_fixed(1, 40000, seed=4, ipv6=True, proto=17)))  # > any fast-lane tile
    recs = rng_recs[:50] + big[:1] + rng_recs[50:120] + big[1:3] + rng_recs[120:] + big[3:]
    pcap = S.build_pcap(recs)
    for args in (["--fixcsum"], ["--seed=3", "--fixcsum"]):
        rc_o, exp = O.rewrite(pcap, args)
        rc, out, r = run(pcap, args)
        assert rc == rc_o == 0 and out == exp
        assert r.fast_lane == 1 and r.generic_tiles >= 1  # the 40000-byte record takes the generic lane


def test_fast_lane_with_tcpprep_cache_directions(built):
    recs = F.mixed(4000, seed=77, near_miss=0.1)
    pcap = F.build(recs)
    cache = S.tcpprep_cache(len(recs), seed=8, nosend_every=13)
    args = ["--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66", "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16",
            "--seed=4", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args, cache)
    rc, out, r = run(pcap, args, cache)
    assert r.fast_lane == 1
    assert rc == rc_o == 0 and out == exp


def test_fast_lane_big_endian_and_nanosecond_input(built):
    recs = F.mixed(1500, seed=9, near_miss=0.0)
    le = F.build(recs)
    args = ["--seed=42", "--fixcsum"]
    _, exp = O.rewrite(le, args)
    # same records as a big-endian nanosecond capture
    be = bytearray(struct.pack(">IHHiIII", 0xA1B23C4D, 2, 4, 0, 0, 65535, 1))
    for ts, tu, cl, ln, d in recs:
        be += struct.pack(">IIII", ts, tu * 1000 + 999, cl, ln) + d
    rc, out, r = run(bytes(be), args)
    assert r.fast_lane == 1 and rc == 0
    assert out == exp


def test_fast_lane_baseline_configs(built):
    for pcap, args in ((S.pcap_fixed(200_000, 64, seed=2), ["--seed=42", "--fixcsum"]),
                       (S.pcap_imix(120_000, seed=3), ["--pnat=10.0.0.0/8:192.168.0.0/16",
                                                      "--portmap=53:5353,80:8080", "--fixcsum"]),
                       (S.pcap_mixed_v4v6(40_000, 1514, seed=5), ["--fixcsum"])):
        rc_o, exp = O.rewrite(pcap, args)
        rc, out, r = run(pcap, args)
        assert r.fast_lane == 1 and r.generic_tiles == 0
        assert rc == rc_o == 0 and out == exp


@pytest.mark.parametrize("near_miss", [0.0, 0.3])
def test_repeat_runs_keep_output_and_counters(built, near_miss):
    """Runs after the first reuse its plan (the generic pass is left out when nothing was
    listed): output, counters and status must not change from run to run."""
    pcap = F.build(F.mixed(3000, seed=21, near_miss=near_miss))
    args = ["--seed=8", "--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=80:8080", "--fixcsum"]
    rc_o, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap)
    try:
        seen = []
        for k in range(4):
            if k == 2:
                b.time(3)  # timed runs in between
            assert b.run() == rc_o
            r = b.result()
            seen.append((b.output(), r.packets, r.bytes_in, r.bytes_out, r.written, r.edited, r.generic_tiles,
                         b.status().tobytes()))
        assert seen[0][0] == exp
        assert all(s == seen[0] for s in seen[1:])
        assert (seen[0][6] == 0) == (near_miss == 0.0)
    finally:
        b.close()
        te.close()
