"""The CPU oracle against the reference's own golden outputs (test/test2.rewrite_*).

This pins the oracle: every in-scope reference golden must be reproduced
byte-for-byte (pcap header included) before the oracle is trusted as the GPU
path's parity checker."""
import pytest

import golden_cases as G
import oracle_lib as O


@pytest.mark.parametrize("case", G.IN_SCOPE, ids=[c[0] for c in G.IN_SCOPE])
def test_oracle_matches_reference_golden(built, case):
    name, inp, cache, args, _ = case
    rc, out = O.rewrite(G.read(inp), args, G.read(cache) if cache else None)
    assert rc == 0
    assert out == G.read(name)


def test_every_reference_golden_is_in_scope():
    assert all(c[4] for c in G.CASES) and len(G.IN_SCOPE) == 33


@pytest.mark.parametrize("args", [["--seed=1", "--fuzz-seed=2"], ["--fuzz-factor=2"], ["--fuzz-seed=1", "--fuzz-factor=0"]])
def test_fuzz_option_constraints(built, args):
    # seed: flags-cant = fuzz-seed; fuzz-factor: flags-must = fuzz-seed, arg-range 1->
    # (src/tcpedit/tcpedit_opts.def:46-48, 324-330)
    with pytest.raises(ValueError):
        O.rewrite(G.read("test.pcap"), args)


def test_seed_mixer_matches_survey_values(built):
    # S(42)=0x75b59d85, S(55)=0xab505be6 (reference tcpr_random)
    assert O.mix_seed(42) == 0x75B59D85
    assert O.mix_seed(55) == 0xAB505BE6


def test_golden_input_checksums(built):
    # only 3 of 179 packets change under --fixcsum
    import tcpreplay_amd.synth as S
    a = S.records(G.read("test.pcap"))
    b = S.records(G.read("test2.rewrite_fixcsum"))
    assert len(a) == len(b) == 179
    changed = [i + 1 for i, (x, y) in enumerate(zip(a, b)) if x != y]
    assert changed == [19, 27, 32]
