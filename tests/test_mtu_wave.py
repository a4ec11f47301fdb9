"""--mtu-trunc on the wave lane (SZ_MTU instances, te_mtu_cuts placement) against the
oracle, bit-exact.

untrunc_packet (edit_packet.c:596-611) cuts a packet longer than l2len + mtu to that
length, sets the IP length fields and, through its return value, forces a checksum
recompute (tcpedit.c:261-265,338).  The wave lane carries plain Ethernet II + IPv4/IPv6
TCP/UDP records; tiles sit at their input offset less the cuts the device predicted for
the records before them, and a tile whose actual output differs from the prediction
(a tagged frame, a record the generic lane treats otherwise) sends the batch to the scan
placement -- the same bytes either way.
"""
import os

import pytest

import fl_cases as F
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu


def run(pcap, args, repeat=1):
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap)
    try:
        outs = []
        for _ in range(repeat):
            rc = b.run()
            outs.append((rc, b.output(), b.result()))
        return outs
    finally:
        b.close()
        te.close()


def first_diff(a, b):
    n = min(len(a), len(b))
    return next((i for i in range(n) if a[i] != b[i]), n)


def check(pcap, args, wave=True, repeat=1):
    rc_o, exp = O.rewrite(pcap, args)
    for rc, out, r in run(pcap, args, repeat):
        assert rc == rc_o
        assert out == exp, f"first difference at byte {first_diff(out, exp)} of {len(exp)}"
        if wave:
            # the wave lane's launch was the last one: the prediction held (no scan rerun)
            assert r.fast_lane == 1
    return exp


@pytest.mark.parametrize("mtu", [128, 296, 576, 1000, 1460, 1500])
def test_mtu_trunc_imix_matches_oracle(built, mtu):
    """IMIX v4 UDP plus 1514-byte v4/v6 TCP/UDP: cuts of every size, records moved by any
    byte count (296: the cut IPv6 payload length is 256, whose raw network-order value
    is below 40 -- edit_packet.c:167 then skips the IPv6 checksum, so those go generic)."""
    recs = (S.records(S.pcap_imix(3000, seed=mtu))
            + S.records(S.pcap_mixed_v4v6(600, size=1514, seed=mtu)))
    recs = [recs[(i * 7919) % len(recs)] for i in range(len(recs))]  # interleave
    check(S.build_pcap(recs), ["--mtu-trunc", f"--mtu={mtu}", "--fixcsum"], wave=mtu != 296)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mtu_trunc_mixed_fast_shapes(built, seed):
    """Random Ethernet II IPv4/IPv6 TCP/UDP records, every size up to 1514."""
    pcap = F.build(F.mixed(5000, seed=300 + seed, near_miss=0.0))
    check(pcap, ["--mtu-trunc", "--mtu=700", "--fixcsum"])


def test_mtu_trunc_without_fixcsum_recomputes(built):
    """untrunc_packet returns 1 for every IP packet, cut or not (edit_packet.c:534,620): a
    run without --fixcsum still recomputes the checksums."""
    pcap = F.build(F.mixed(4000, seed=41, near_miss=0.0))
    check(pcap, ["--mtu-trunc", "--mtu=900"])


@pytest.mark.parametrize("seed", [5, 6])
def test_mtu_trunc_near_misses(built, seed):
    """A quarter of the records are shapes the wave lane leaves to the generic lane
    (tags, IP options, fragments, padding, extension headers, ICMP, ARP, snaplen-cut
    captures, len != caplen): their tiles are redone there at the predicted offsets."""
    pcap = F.build(F.mixed(6000, seed=400 + seed, near_miss=0.25))
    check(pcap, ["--mtu-trunc", "--mtu=600", "--fixcsum"], wave=False)


@pytest.mark.parametrize("args", [
    ["--seed=42"],
    ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080"],
    ["--enet-dmac=00:12:13:14:15:16", "--enet-smac=00:22:33:44:55:66", "--ttl=+3", "--tos=9"],
    ["--pnat=[2001::/16]:[2001:db8:aaaa::/48],[2606::/16]:[fd00::/8]", "--tclass=5", "--flowlabel=77"],
])
def test_mtu_trunc_with_other_edits(built, args):
    pcap = F.build(F.mixed(4000, seed=77, near_miss=0.0))
    check(pcap, args + ["--mtu-trunc", "--mtu=800", "--fixcsum"])


def test_mtu_trunc_repeat_runs_and_tagged_fallback(built):
    """Repeat runs of one batch keep their bytes; a capture of tagged frames (predicted
    l2len 18, generic lane) and untagged ones in one batch."""
    plain = S.records(S.pcap_imix(2000, seed=8))
    tagged = S.records(S.pcap_imix(300, seed=9, vlan=0x0064))
    recs = plain[:900] + tagged + plain[900:]
    check(S.build_pcap(recs), ["--mtu-trunc", "--mtu=1000", "--fixcsum"], wave=False, repeat=3)
    check(S.build_pcap(plain), ["--mtu-trunc", "--mtu=1000", "--fixcsum"], repeat=3)


def test_mtu_trunc_scan_placement_agrees(built):
    """The wave lane's output equals the generic lane's (TCPEDIT_HIP_NO_MTU_FAST=1)."""
    pcap = F.build(F.mixed(5000, seed=91, near_miss=0.1))
    args = ["--mtu-trunc", "--mtu=500", "--fixcsum"]
    a = run(pcap, args)[0]
    os.environ["TCPEDIT_HIP_NO_MTU_FAST"] = "1"
    try:
        b = run(pcap, args)[0]
    finally:
        del os.environ["TCPEDIT_HIP_NO_MTU_FAST"]
    assert a[0] == b[0] and a[1] == b[1]
    assert b[2].fast_lane == 0


def test_mtu_trunc_large_batch(built):
    """A batch of many wave rounds (300K IMIX records): byte-exact against the oracle."""
    pcap = S.pcap_imix(300000, seed=12)
    check(pcap, ["--mtu-trunc", "--mtu=1000", "--fixcsum"])
