"""tcpreplay-edit's tcpedit calls, batched (tcpedit_replay_* in include/tcpedit.h).

tcpreplay-edit edits every record it sends with tcpedit_packet (send_packets.c:469-474)
and, with -K (--preload-pcap), edits the cached copy IN PLACE on every pass after the
first, so edits compound from one --loop pass to the next.  The oracle
restates that loop with file output (tcpreplay_edit_oracle_run); the reference holds no
tcpreplay-edit output fixture, so the loop itself is "parity unpinned" -- but a single
pass edits each record exactly as tcprewrite does, and that is pinned against the
reference's tcprewrite goldens (test2.*) below.

CPU tests: the oracle against the goldens and the compounding rules; GPU tests: the
library (Python mirror and the relinked C caller tests/abi/tcpreplay_edit_abi.c)
against the oracle, bit-exact.
"""
import os
import struct
import subprocess

import pytest

import golden_cases as G
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABI_DIR = os.path.join(ROOT, "tests", "abi")
ABI_BIN = os.path.join(ABI_DIR, "_build", "tcpreplay_edit_abi")

# tcprewrite-only options (not tcpedit's): cases using them have no tcpreplay-edit analogue
# (--fuzz-seed is tcpedit's, tcpreplay_opts.def:572: its passes are below)
_TCPREWRITE_ONLY = ("--skip-soft-errors", "--dlt=")


def _edit_cases():
    return [c for c in G.IN_SCOPE if not c[2] and not any(a.startswith(_TCPREWRITE_ONLY) for a in c[3])]


# the reference's tcpreplay goldens of the per-pass packet list (test/Makefile.am:214-215):
# tcpreplay-edit with no tcpedit option writes what tcpreplay writes
LIST_GOLDENS = [("test2.replay_include", ["--include=7,11,20-23,174-"]),
                ("test2.replay_exclude", ["--exclude=23-,11-20,2,3"])]


def _recs(dump: bytes):
    """(ts_sec, frac, caplen, len, data) of a dump's records"""
    out, p = [], 24
    while p + 16 <= len(dump):
        ts, fr, cl, ln = struct.unpack_from("<IIII", dump, p)
        out.append((ts, fr, cl, ln, dump[p + 16:p + 16 + cl]))
        p += 16 + cl
    assert p == len(dump)
    return out


def _passes(dump: bytes, loops: int):
    r = _recs(dump)
    n = len(r) // loops
    assert n * loops == len(r)
    return [r[i * n:(i + 1) * n] for i in range(loops)]


# ---------------------------------------------------------------- the oracle (CPU)
@pytest.mark.parametrize("case", _edit_cases(), ids=lambda c: c[0])
def test_one_pass_edits_as_tcprewrite_does(case):
    """one pass edits every record exactly as tcprewrite (the reference's goldens); the
    -w dump carries libpcap's nanosecond fraction (x1000 for a microsecond capture) and
    pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN)'s header"""
    name, inp, _, args, _ = case
    rc, dump = O.replay_edit(G.read(inp), args)
    assert rc == 0
    assert dump[:24] == TA.REPLAY_DUMP_HEADER
    gold = S.records(G.read(name))
    # (a record the fuzz step emptied: pcap_dump writes it, tcprewrite.c:367 does not; no
    # record is read with caplen 0 -- safe_pcap_next exits there, utils.c:147-156)
    got = [r for r in _recs(dump) if r[2]]
    assert len(got) == len(gold)
    for (ts, fr, cl, ln, d), (gts, gtu, gcl, gln, gd) in zip(got, gold):
        assert (ts, fr, cl, ln, d) == (gts, gtu * 1000, gcl, gln, gd)


def test_preload_compounds_vlan_add_from_the_third_pass():
    """-K: pass 0 edits libpcap's buffer and caches the unedited bytes; pass 1 edits the
    cache (unedited: same output); pass 2 edits what pass 1 left in it with the cached
    (original) header -- a second 802.1Q tag, the record's last 4 bytes gone"""
    pcap = S.pcap_fixed(50, 90, seed=3)
    args = ["--enet-vlan=add", "--enet-vlan-tag=7", "--enet-vlan-pri=1"]
    rc, dump = O.replay_edit(pcap, args, loops=3, preload=True)
    assert rc == 0
    p0, p1, p2 = _passes(dump, 3)
    assert p0 == p1
    for a, b in zip(p1, p2):
        assert b[2] == a[2] and b[3] == a[3]  # caplen, len: original + 4 both times
        tag = a[4][12:16]
        assert tag[:2] == b"\x81\x00" and b[4][12:16] == tag and b[4][16:20] == tag
        assert b[4][20:] == a[4][16:-4]
    # without -K every pass reads the file again: no compounding
    rc, dump = O.replay_edit(pcap, args, loops=3)
    q0, q1, q2 = _passes(dump, 3)
    assert q0 == q1 == q2 == p0


def test_preload_compounds_efcs():
    """--efcs under -K strips 4 more bytes of the cached record every pass after the
    first (the cached header's caplen stays the original)"""
    pcap = S.pcap_imix(400, seed=5, fcs=True)
    rc, dump = O.replay_edit(pcap, ["--efcs"], loops=3, preload=True)
    assert rc == 0
    p0, p1, p2 = _passes(dump, 3)
    assert p0 == p1
    for a, b in zip(p1, p2):
        assert b[2] == a[2] and b[4] == a[4][:b[2]]


@pytest.mark.parametrize("name,args", LIST_GOLDENS)
def test_oracle_list_pass_is_the_reference_golden(name, args):
    """send_packets.c:440-447 before tcpedit_packet: pinned by the reference's goldens"""
    rc, dump = O.replay_edit(G.read("test.pcap"), args)
    assert rc == 0 and dump == G.read(name)


def test_oracle_list_and_unique_ip_ride_the_edit_pass():
    """one pass carries the list, the edit and fast_edit_packet (:440-483): listed-out
    records are neither edited nor sent; the edited records of the passes where
    unique_iteration advanced get their addresses shifted after the edit"""
    pcap = G.read("test.pcap")
    rc, dump = O.replay_edit(pcap, ["--include=1-100", "--unique-ip", "--seed=5"], loops=2)
    assert rc == 0
    failed = O.replay_edit_failed()
    assert failed > 0  # test.pcap's non-IP records among the first 100
    p0, p1 = _passes_n(dump, [100, 100 - failed])
    rc, one = O.replay_edit(pcap, ["--include=1-100", "--seed=5"])
    assert p0 == _recs(one)
    assert len(p1) == 100 - failed


def _passes_n(dump, counts):
    r, out, i = _recs(dump), [], 0
    for c in counts:
        out.append(r[i:i + c])
        i += c
    assert i == len(r)
    return out


def test_fuzz_with_preload_is_refused():
    with pytest.raises(ValueError):
        O.replay_edit(S.pcap_fixed(10, 64, seed=1), ["--fuzz-seed=3"], loops=2, preload=True)


def test_hard_error_ends_the_run_with_the_records_sent_before():
    recs = S.records(G.read("test.pcap"))[:10]
    ts, tu, cl, ln, d = recs[4]
    d = bytearray(d)
    d[14] = 0x55  # IP version 5 under ethertype IPv4 (edit_packet.c:73-79)
    recs[4] = (ts, tu, cl, ln, bytes(d))
    rc, dump = O.replay_edit(S.build_pcap(recs), ["--fixcsum"], loops=2)
    assert rc == -1 and len(_recs(dump)) == 4


# ---------------------------------------------------------------- the device (GPU)
def _synth_cases():
    return [
        ("c2", lambda: S.pcap_fixed(20_000, 64, seed=21), ["--seed=42", "--fixcsum"]),
        ("imix", lambda: S.pcap_imix(6_000, seed=22), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353",
                                                      "--fixcsum"]),
        ("vlan", lambda: S.pcap_imix(3_000, seed=23), ["--enet-vlan=add", "--enet-vlan-tag=45", "--fixcsum"]),
        ("vlandel", lambda: S.pcap_imix(3_000, seed=26, vlan=12), ["--enet-vlan=del", "--fixcsum"]),
        ("efcs", lambda: S.pcap_imix(3_000, seed=24, fcs=True), ["--efcs", "--ttl=3"]),
        ("mtu", lambda: S.pcap_imix(3_000, seed=25), ["--mtu=300", "--mtu-trunc", "--fixcsum"]),
        ("pad", lambda: S.pcap_imix(3_000, seed=27), ["--fixlen=pad", "--fixcsum"]),
        ("macseed", lambda: S.pcap_fixed(5_000, 128, seed=28), ["--enet-mac-seed=9", "--fixcsum"]),
    ]


@pytest.mark.gpu
@pytest.mark.parametrize("loops,preload", [(1, False), (3, False), (3, True)])
@pytest.mark.parametrize("name,gen,args", _synth_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_replay_passes_match_the_oracle(built, name, gen, args, loops, preload):
    pcap = gen()
    rc_o, exp = O.replay_edit(pcap, args, loops, preload)
    errs = []
    rc, out = TA.replay_edit(pcap, args, loops, preload, errors=errs)
    assert rc == rc_o == 0, errs
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"


def _cached_image(pcap, pass_recs):
    """the -K cache after a cached pass: each record's edited bytes (up to its original
    caplen), then the bytes the edit did not reach, behind the file's own headers"""
    parts, recs = [pcap[:24]], S.records(pcap)
    for (ts, tu, cl, ln, d0), r in zip(recs, pass_recs):
        d1 = r[4]
        n = min(len(d1), cl)
        parts.append(struct.pack("<IIII", ts, tu, cl, ln) + d1[:n] + d0[n:cl])
    return b"".join(parts)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["vlandel", "vlan", "efcs"])
def test_cached_pass_image_rewrites_as_the_oracle(built, name):
    """a cached pass is a batch over the cache image: the batch path alone on that image"""
    case = next(c for c in _synth_cases() if c[0] == name)
    pcap, args = case[1](), case[2]
    rc, dump = O.replay_edit(pcap, args, 2, True)
    img = _cached_image(pcap, _passes(dump, 2)[1])
    rc_o, exp = O.rewrite(img, args)
    te = TA.TcpEdit(args)
    try:
        rc_g, out = te.rewrite(img)
        err = te.geterr()
    finally:
        te.close()
    assert rc_g == rc_o, err
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", _edit_cases(), ids=lambda c: c[0])
def test_replay_over_the_goldens_matches_the_oracle(built, case):
    name, inp, _, args, _ = case
    pcap = G.read(inp)
    fuzz = any(a.startswith("--fuzz-seed") for a in args)
    for loops, preload in ((1, False), (2, not fuzz)):  # (--fuzz-seed with -K: refused by both)
        rc_o, exp = O.replay_edit(pcap, args, loops, preload)
        rc, out = TA.replay_edit(pcap, args, loops, preload)
        assert (rc, out) == (rc_o, exp)


@pytest.mark.gpu
def test_replay_hard_error_matches_the_oracle(built):
    recs = S.records(G.read("test.pcap"))[:10]
    ts, tu, cl, ln, d = recs[4]
    d = bytearray(d)
    d[14] = 0x55
    recs[4] = (ts, tu, cl, ln, bytes(d))
    pcap = S.build_pcap(recs)
    rc_o, exp = O.replay_edit(pcap, ["--fixcsum"], 2)
    rc, out = TA.replay_edit(pcap, ["--fixcsum"], 2)
    assert rc_o == -1 and rc == TA.TCPEDIT_ERROR and out == exp


@pytest.mark.gpu
@pytest.mark.parametrize("loops,preload", [(1, False), (3, False), (3, True)])
def test_replay_reader_rules_match_the_oracle(built, loops, preload):
    """safe_pcap_next (send_packets.c:955,985 -> src/common/utils.c:131-169): len < caplen
    records are edited and sent as len bytes (and cached so under -K); a zero len or caplen
    record ends the run in the first pass, after the records before it were sent"""
    recs = S.records(S.pcap_imix(3000, seed=21))
    for i in range(5, len(recs), 41):
        ts, tu, cl, ln, d = recs[i]
        recs[i] = (ts, tu, cl, max(1, cl - 1 - i % 50), d)
    args = ["--enet-vlan=add", "--enet-vlan-tag=9", "--seed=4", "--fixcsum"]
    pcap = S.build_pcap(recs)
    rc_o, exp = O.replay_edit(pcap, args, loops, preload)
    rc, out = TA.replay_edit(pcap, args, loops, preload)
    assert rc_o == 0 and rc == 0 and out == exp
    for zc, zl in ((0, 0), (0, 90), (90, 0)):
        ts, tu, cl, ln, d = recs[2222]
        bad = S.build_pcap(recs[:2222] + [(ts, tu, zc, zl, d[:zc])] + recs[2223:])
        rc_o, exp = O.replay_edit(bad, args, loops, preload)
        rc, out = TA.replay_edit(bad, args, loops, preload)
        assert rc_o == -1 and rc == TA.TCPEDIT_ERROR and out == exp


@pytest.fixture(scope="module")
def abi(built):
    import fcntl
    os.makedirs(os.path.join(ABI_DIR, "_build"), exist_ok=True)
    with open(os.path.join(ABI_DIR, "_build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            subprocess.check_call(["make", "-s", "-C", ABI_DIR])
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return ABI_BIN


@pytest.mark.gpu
@pytest.mark.parametrize("loops,preload,extra", [(1, False, []), (4, True, []),
                                                 (3, True, ["--exclude=100-200,3000-", "--unique-ip"])])
def test_relinked_tcpreplay_edit_writes_the_oracle_dump(abi, tmp_path, loops, preload, extra):
    """tcpreplay.c:79-100's calls and the send loop through the C-ABI caller, -w file"""
    pcap = S.pcap_imix(4_000, seed=31)
    args = ["--enet-vlan=add", "--enet-vlan-tag=9", "--pnat=10.0.0.0/8:172.16.0.0/12", "--fixcsum"] + extra
    inp, out = tmp_path / "in.pcap", tmp_path / "out.pcap"
    inp.write_bytes(pcap)
    cmd = [abi, "-w", str(out), f"--loop={loops}"] + (["-K"] if preload else []) + args + [str(inp)]
    r = subprocess.run(cmd, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    rc_o, exp = O.replay_edit(pcap, args, loops, preload)
    assert rc_o == 0 and out.read_bytes() == exp


# --------------------------------------- the pass's other steps: the list and --unique-ip
REPLAY_LINES = [
    (["--include=7,11,20-23,174-"], 1, False),
    (["--exclude=23-,11-20,2,3", "--seed=9", "--fixcsum"], 2, False),
    (["--include=1-1500,2500-", "--unique-ip", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"], 3, False),
    (["--exclude=5-40", "--unique-ip", "--enet-vlan=add", "--enet-vlan-tag=7", "--fixcsum"], 3, True),
    (["--unique-ip", "--unique-ip-loops=2", "--ttl=+3"], 5, True),
    (["--include=2-", "--unique-ip", "--efcs"], 3, True),
    (["--fuzz-seed=42", "--fuzz-factor=2"], 3, False),  # the RNG stream runs on across passes
    (["--exclude=1-999", "--fuzz-seed=7", "--fuzz-factor=1", "--unique-ip"], 3, False),  # no draws for them
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,args", LIST_GOLDENS)
def test_replay_list_reproduces_the_reference_golden(built, name, args):
    rc, out = TA.replay_edit(G.read("test.pcap"), args)
    assert rc == 0 and out == G.read(name)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(REPLAY_LINES)))
def test_replay_list_unique_ip_and_fuzz_match_the_oracle(built, k):
    args, loops, preload = REPLAY_LINES[k]
    for pcap in (G.read("test.pcap"), S.pcap_imix(5_000, seed=40 + k)):
        rc_o, exp = O.replay_edit(pcap, args, loops, preload)
        failed_o = O.replay_edit_failed()
        rargs, eargs = TA.split_replay_args(args)
        te = TA.TcpEdit(eargs)
        try:
            r = TA.Replay(te, pcap, preload, rargs)
            out = [TA.REPLAY_DUMP_HEADER]
            for _ in range(loops):
                rc, recs = r.pass_()
                out.append(recs)
            assert rc == rc_o == 0, te.geterr()
            assert b"".join(out) == exp
            assert r.failed == failed_o
            r.close()
        finally:
            te.close()
