"""--fuzz-seed on the wave lane (te_launch_t.static_fz): the header reach kernel
(te_fuzz_reach) plus the generic reach pass over the tiles it lists, the RNG states,
the predicted per-tile cuts (te_fuzz_tile_cut), and the wave lane's fuzz step and
cut store (SZ_FUZZ) -- bit-exact against the oracle (fuzzing.c:80-199 through
tcpedit.c:250-258), and record for record against the generic lane
(TCPEDIT_HIP_NO_FUZZ_FAST=1), counters included."""
import os

import pytest

import fl_cases as F
import golden_cases as G
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu

# configs the wave lane fuzzes: no edit before the fuzz step (fast_capable_fuzz)
FZ_SETS = [
    ["--fuzz-seed=42", "--fuzz-factor=2"],
    ["--fuzz-seed=7", "--fuzz-factor=1", "--fixcsum"],
    ["--fuzz-seed=1"],
    ["--fuzz-seed=3", "--fuzz-factor=1", "--srcipmap=0.0.0.0/0:10.1.0.0/16"],
    ["--fuzz-seed=5", "--fuzz-factor=2", "--pnat=10.0.0.0/8:192.168.0.0/16", "--fixcsum"],
    ["--fuzz-seed=8", "--fuzz-factor=1", "--pnat=[2001::/16]:[fd00::/8]"],
    ["--fuzz-seed=4242", "--fuzz-factor=3", "--skipbroadcast", "--dstipmap=10.0.0.0/8:172.16.0.0/12", "--fixcsum"],
]
# (--seed and --fuzz-seed are mutually exclusive options)
COUNTERS = ("packets", "bytes_in", "bytes_out", "written", "edited", "soft_errors", "warnings", "errors")


def run(pcap, args, generic=False):
    if generic:
        os.environ["TCPEDIT_HIP_NO_FUZZ_FAST"] = "1"
    try:
        te = TA.TcpEdit(args)
        b = TA.Batch(te, pcap)
        try:
            rc = b.run()
            return rc, b.output(), b.result(), b.status()
        finally:
            b.close()
            te.close()
    finally:
        os.environ.pop("TCPEDIT_HIP_NO_FUZZ_FAST", None)


def first_diff(a, b):
    n = min(len(a), len(b))
    return next((i for i in range(n) if a[i] != b[i]), n)


def check(pcap, args, all_wave=False):
    rc_o, exp = O.rewrite(pcap, args)
    rc, out, r, st = run(pcap, args)
    assert r.fast_lane == 1
    if all_wave:
        assert r.generic_tiles == 0
    assert rc == rc_o
    assert out == exp, f"first difference at byte {first_diff(out, exp)}"
    rc2, out2, r2, st2 = run(pcap, args, generic=True)
    assert r2.fast_lane == 0 and rc2 == rc and out2 == out
    assert [getattr(r, k) for k in COUNTERS] == [getattr(r2, k) for k in COUNTERS]
    assert (st == st2).all()
    return r


@pytest.mark.parametrize("k", range(len(FZ_SETS)))
def test_fuzz_wave_mixed_shapes(built, k):
    """The fast-lane shapes with the near misses the generic lane takes (their tiles are
    reach-listed, then redone by the generic lane from the same states)."""
    check(F.build(F.mixed(6000, seed=300 + k)), FZ_SETS[k])


@pytest.mark.parametrize("k", [0, 1, 3, 5])
def test_fuzz_wave_pure_shapes_stay_on_the_wave_lane(built, k):
    """Every record of a wave-lane shape: nothing listed for either the reach pass or the
    edit, DROP / REDUCE / byte runs all on the wave lane."""
    r = check(F.build(F.mixed(4000, seed=17 + k, near_miss=0.0)), FZ_SETS[k], all_wave=True)
    assert r.soft_errors > 0  # (the cuts happened)
    assert r.written < r.packets  # (and some were drops)


def test_fuzz_wave_imix_and_golden(built):
    gold = S.records(G.read("test.pcap"))
    recs = S.records(S.pcap_imix(20_000, seed=5)) + gold + S.records(S.pcap_fixed(3000, 60, seed=6))
    check(S.build_pcap(recs), ["--fuzz-seed=42", "--fuzz-factor=2"])


def test_fuzz_wave_l7fuzzing_golden(built):
    rc, out, r, _ = run(G.read("test.pcap"), ["--fuzz-seed=42", "--fuzz-factor=2"])
    assert rc == 0 and r.fast_lane == 1
    assert S.records(out) == S.records(G.read("test2.rewrite_l7fuzzing"))


def test_fuzz_wave_state_continues_across_runs(built):
    """The context's RNG state after a wave-lane run is the state after its reaching
    records: a second batch continues the stream (== one oracle run over both)."""
    args = ["--fuzz-seed=99", "--fuzz-factor=2", "--fixcsum"]
    recs = S.records(F.build(F.mixed(5000, seed=61)))
    rc_o, exp = O.rewrite(S.build_pcap(recs), args)
    te = TA.TcpEdit(args)
    try:
        outs = []
        for part in (recs[:2222], recs[2222:]):
            b = TA.Batch(te, S.build_pcap(part))
            try:
                assert b.run() == 0
                assert b.result().fast_lane == 1
                outs += S.records(b.output())
            finally:
                b.close()
    finally:
        te.close()
    assert rc_o == 0 and outs == S.records(exp)


def test_fuzz_wave_a_million_records(built):
    """> 2^20 records: many reach / cut blocks, the state scan's loop."""
    pcap = S.pcap_imix(1_100_000, seed=33)
    check(pcap, ["--fuzz-seed=77", "--fuzz-factor=3", "--fixcsum"])
