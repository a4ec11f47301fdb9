"""Static +-4 placement falling back to scan + look-back.

A VLAN pop or --efcs as the only size change places record i at its input offset - 4 i;
a record that does not shrink by exactly 4 (an untagged record under --enet-vlan=del)
sets the violation word and the host places the batch again by scan and look-back.
These cases reach that fallback on a fresh batch and on a batch whose earlier runs
placed statically (tcpreplay-edit's -K passes re-run one batch over updated bytes,
te_replay.c).  GPU = oracle, bit-exact."""
import struct

import pytest

import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S


def _untag_keep_len(pcap, every=1):
    """every `every`-th tagged record rewritten as the -K cache holds it after a VLAN pop:
    the untagged frame, then the record's last 4 original bytes (caplen unchanged)"""
    parts = [pcap[:24]]
    for i, (ts, tu, cl, ln, d) in enumerate(S.records(pcap)):
        if i % every == 0 and d[12:14] == b"\x81\x00":
            d = d[:12] + d[16:] + d[-4:]
        parts.append(struct.pack("<IIII", ts, tu, cl, ln) + d)
    return b"".join(parts)


ARGS = ["--enet-vlan=del", "--fixcsum"]


@pytest.mark.gpu
@pytest.mark.parametrize("every", [1, 3, 1000])
def test_fresh_batch_with_untagged_records(built, every):
    pcap = _untag_keep_len(S.pcap_imix(3_000, seed=31, vlan=12), every)
    rc_o, exp = O.rewrite(pcap, ARGS)
    te = TA.TcpEdit(ARGS)
    try:
        b = TA.Batch(te, pcap)
        assert b.run() == 0, te.geterr()
        assert b.output() == exp
        b.close()
    finally:
        te.close()


@pytest.mark.gpu
@pytest.mark.parametrize("every", [1, 3])
def test_static_batch_updated_to_untagged_records(built, every):
    tagged = S.pcap_imix(3_000, seed=32, vlan=12)
    mixed = _untag_keep_len(tagged, every)
    te = TA.TcpEdit(ARGS)
    try:
        b = TA.Batch(te, tagged)
        for img in (tagged, tagged, mixed, mixed, tagged):
            b.update_input(img)
            assert b.run() == 0, te.geterr()
            rc_o, exp = O.rewrite(img, ARGS)
            assert rc_o == 0
            got = b.output()
            assert got == exp, f"first difference at byte {next((i for i in range(min(len(got), len(exp))) if got[i] != exp[i]), min(len(got), len(exp)))} ({len(got)} vs {len(exp)})"
        b.close()
    finally:
        te.close()
