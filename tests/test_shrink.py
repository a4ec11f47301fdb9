"""The wave lane's size-reducing edits, bit-exact against the oracle:

  --enet-vlan=del over single-tagged records (dlt_en10mb_encode's pop, en10mb.c:520-578)
  --efcs over frames that carry an FCS (tcpedit.c:78-84)

Every record then shrinks by 4 bytes, so outputs sit at input offset - 4 x index (static
placement, no scan) and the wave lane drops the 4 bytes in its store.  A capture that
breaks the placement (an untagged record under the pop, caplen != len under --efcs, a
hard error) is placed by scan + look-back instead; the bytes must not change either way.
"""
import struct

import pytest

import fl_cases as F
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu

EDIT_SETS = [
    ["--fixcsum"],
    ["--seed=42", "--fixcsum"],
    ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"],
    ["--pnat=[2001::/16]:[2001:db8:aaaa::/48],[2606::/16]:[fd00::/8]", "--fixcsum"],
    ["--enet-dmac=00:12:13:14:15:16", "--enet-smac=00:22:33:44:55:66", "--skipl2broadcast", "--fixcsum"],
    ["--seed=7", "--ttl=+3", "--tos=7"],  # incremental checksums, a recomputation on TTL change
    ["--tcp-sequence=77", "--flowlabel=5", "--tclass=3", "--portmap=1-65535:7"],
]


def tag(recs, tpids=(0x8100,), every=1):
    """a {TPID, TCI} tag after the MACs of every `every`-th record"""
    out = []
    for i, (ts, tu, cl, ln, d) in enumerate(recs):
        if i % every == 0 and cl >= 14:
            t = struct.pack("!HH", tpids[i % len(tpids)], (i * 2654435761) & 0xFFFF)
            d = d[:12] + t + d[12:]
            cl, ln = cl + 4, ln + 4
        out.append((ts, tu, cl, ln, d))
    return out


def fcs(recs, every=1):
    """4 trailing FCS bytes on every `every`-th record (caplen and len both count them)"""
    out = []
    for i, (ts, tu, cl, ln, d) in enumerate(recs):
        if i % every == 0 and cl == ln:
            d = d + struct.pack("<I", (i * 2246822519) & 0xFFFFFFFF)
            cl, ln = cl + 4, ln + 4
        out.append((ts, tu, cl, ln, d))
    return out


def corrupt(recs):
    """every IPv4 header checksum and TCP / UDP checksum (a zero UDP one aside) made wrong:
    --fixcsum must then recompute them all, where incremental updates would carry the
    error along"""
    out = []
    for ts, tu, cl, ln, d in recs:
        d = bytearray(d)
        et = d[12:14]
        l4, proto = (34, d[23]) if et == b"\x08\x00" else (54, d[20]) if et == b"\x86\xdd" else (None, None)
        if l4 is not None:
            if et == b"\x08\x00":
                d[24] ^= 0x5A
            f = l4 + (16 if proto == 6 else 6)
            if f + 2 <= cl and (proto == 6 or d[f:f + 2] != b"\0\0"):
                d[f] ^= 0xA5
        out.append((ts, tu, cl, ln, bytes(d)))
    return out


def run_twice(pcap, args):
    """two runs of one batch (the second leaves the generic pass out when the first listed
    no tile); returns the return code, output and result of the first"""
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap)
        rc = b.run()
        out, r = b.output(), b.result()
        rc2 = b.run()
        assert rc2 == rc and b.output() == out
        b.close()
        return rc, out, r
    finally:
        te.close()


def check(pcap, args, pure):
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, r = run_twice(pcap, args)
    assert rc == rc_o
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"
    if rc_o == 0:
        assert r.bytes_out == len(exp) - 24
    if pure:  # every record a fast shape: the wave lane finishes every tile
        assert r.fast_kind == 2 and r.generic_tiles == 0
    return r


@pytest.mark.parametrize("k", range(len(EDIT_SETS)))
def test_vlan_pop_on_the_wave_lane(built, k):
    pcap = F.build(tag(F.mixed(3000, seed=300 + k, near_miss=0.0), tpids=(0x8100, 0x88A8, 0x9100)))
    check(pcap, ["--enet-vlan=del"] + EDIT_SETS[k], pure=True)


@pytest.mark.parametrize("k", range(len(EDIT_SETS)))
def test_efcs_on_the_wave_lane(built, k):
    pcap = F.build(fcs(F.mixed(3000, seed=400 + k, near_miss=0.0)))
    check(pcap, ["--efcs"] + EDIT_SETS[k], pure=True)


@pytest.mark.parametrize("seed", range(3))
def test_vlan_pop_near_misses(built, seed):
    """tagged near-miss shapes (a second tag, IP options, fragments, ARP, truncations,
    len != caplen): the wave lane lists their tiles, the generic lane writes them at the
    same static offsets (or the batch is placed by scan when one does not shrink)"""
    pcap = F.build(tag(F.mixed(4000, seed=500 + seed, near_miss=0.25)))
    check(pcap, ["--enet-vlan=del", "--seed=3", "--fixcsum"], pure=False)


@pytest.mark.parametrize("seed", range(3))
def test_efcs_near_misses(built, seed):
    pcap = F.build(fcs(F.mixed(4000, seed=600 + seed, near_miss=0.25)))
    check(pcap, ["--efcs", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"], pure=False)


def test_vlan_pop_with_untagged_records_falls_back_to_scan(built):
    """every third record untagged: it keeps its size, the static placement breaks and the
    batch is placed by scan"""
    pcap = F.build(tag(F.mixed(3000, seed=71, near_miss=0.0), every=3))
    check(pcap, ["--enet-vlan=del", "--fixcsum"], pure=False)


def test_efcs_with_len_caplen_mismatch_falls_back_to_scan(built):
    """records without an FCS among FCS frames, and one snaplen-cut record (--efcs keeps its
    caplen, reduces its len)"""
    recs = fcs(F.mixed(3000, seed=72, near_miss=0.0), every=2)
    ts, tu, cl, ln, d = recs[1500]
    recs[1500] = (ts, tu, cl - 10, ln, d[:cl - 10])
    check(F.build(recs), ["--efcs", "--seed=1", "--fixcsum"], pure=False)


@pytest.mark.parametrize("args,kw", [
    (["--enet-vlan=del", "--fixcsum"], dict(vlan=0xB02D)),
    (["--efcs", "--fixcsum"], dict(fcs=True)),
    (["--enet-vlan=del", "--seed=42", "--portmap=53:5353"], dict(vlan=7)),
    (["--efcs", "--seed=42", "--ttl=9"], dict(fcs=True)),
], ids=["vdel", "efcs", "vdel-incr", "efcs-incr"])
def test_shrink_bench_workloads(built, args, kw):
    """the bench's vdel / efcs IMIX workloads (64/570/1514 7:4:1) at 120k records"""
    check(S.pcap_imix(120_000, seed=5, **kw), args, pure=True)


@pytest.mark.parametrize("shape", ["none", "vdel", "efcs"])
def test_fixcsum_recomputes_wrong_checksums_with_header_edits(built, shape):
    """--fixcsum with an IP header edit and MAC / port / address edits (the widest wave-lane
    instance that is not incremental) on records whose checksums are all wrong"""
    recs = corrupt(F.mixed(3000, seed=74, near_miss=0.0))
    extra = {"none": [], "vdel": ["--enet-vlan=del"], "efcs": ["--efcs"]}[shape]
    recs = tag(recs) if shape == "vdel" else fcs(recs) if shape == "efcs" else recs
    args = extra + ["--tos=9", "--enet-smac=00:22:33:44:55:66", "--portmap=53:5353",
                    "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"]
    check(F.build(recs), args, pure=True)
    check(F.build(recs), extra + ["--tos=9", "--fixcsum"], pure=True)


def test_efcs_and_vlan_pop_together_stay_generic(built):
    """both size changes at once (-8 a record) are not a static placement: scan"""
    pcap = F.build(fcs(tag(F.mixed(1500, seed=73, near_miss=0.0))))
    check(pcap, ["--efcs", "--enet-vlan=del", "--fixcsum"], pure=False)
