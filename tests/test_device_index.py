"""The record index built on the device (te_index.hip, tcpedit_batch_index_device):
windows of the capture, speculative record-boundary guesses per lane checked against
the chain, the wave-lane tile cut.  Every case runs the edit with the device-built index
and must write the oracle's bytes; where the speculation is fooled (record-like bytes in
payloads) the batch keeps the host walk's index, and the bytes must not change either."""
import struct

import pytest

import fl_cases as F
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

pytestmark = pytest.mark.gpu


def _run(pcap, args, cache=None, expect_applied=True):
    rc_o, exp = O.rewrite(pcap, args, cache)
    te = TA.TcpEdit(args)
    try:
        b = TA.Batch(te, pcap, cache)
        host_tiles = b.result().n_tiles if hasattr(b.result(), "n_tiles") else None
        applied, ms = b.index_device(iters=2)
        if expect_applied is not None:
            assert applied == expect_applied
        rc = b.run()
        out, r = b.output(), b.result()
        b.close()
    finally:
        te.close()
    assert rc == rc_o
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"
    return applied, ms, r, host_tiles


@pytest.mark.parametrize("name,gen,args", [
    ("c2", lambda: S.pcap_fixed(100_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
    ("imix", lambda: S.pcap_imix(60_000, seed=2), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353",
                                                   "--fixcsum"]),
    ("mixed", lambda: F.build(F.mixed(8000, seed=3)), ["--seed=7", "--fixcsum"]),
    ("vlan-add", lambda: S.pcap_imix(30_000, seed=4), ["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"]),
    ("vlan-del", lambda: S.pcap_imix(30_000, seed=5, vlan=9), ["--enet-vlan=del", "--fixcsum"]),
    ("efcs", lambda: S.pcap_imix(30_000, seed=6, fcs=True), ["--efcs", "--ttl=3"]),
    ("c5", lambda: S.pcap_mixed_v4v6(20_000, 1514, seed=7), ["--fixcsum"]),
], ids=lambda x: x if isinstance(x, str) else "")
def test_device_index_matches_the_host_walk(built, name, gen, args):
    applied, ms, r, _ = _run(gen(), args)
    assert applied and ms > 0


def test_device_index_with_a_tcpprep_cache(built):
    pcap = S.pcap_imix(40_000, seed=8)
    cache = S.tcpprep_cache(40_000, seed=8, nosend_every=7)
    args = ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66", "--fixcsum"]
    _run(pcap, args, cache)


def test_tiny_huge_and_trimmed_records(built):
    """caplen 1..21 records (the fast lane defers them), records larger than a wave tile
    (solo) and than a generic slot (huge: HBM scratch), and len < caplen records (the
    reader trims caplen to len, src/common/utils.c:159-162), between ordinary ones"""
    base = S.records(S.pcap_fixed(3000, 90, seed=9))
    big = S.records(S.pcap_fixed(3, 9000, seed=10)) + S.records(S.pcap_fixed(2, 40000, seed=11))
    recs = []
    for i, r in enumerate(base):
        recs.append(r)
        if i % 97 == 0:
            recs.append((1, i, 1 + i % 21, 1 + i % 21, bytes(1 + i % 21)))
        if i % 89 == 5:
            ts, tu, cl, ln, d = r
            recs.append((ts, tu, cl, cl - 1 - i % 40, d))
        if i % 701 == 0:
            recs.append(big[(i // 701) % len(big)])
    _run(S.build_pcap(recs), ["--seed=3", "--fixcsum"])


def test_the_chain_ends_as_libpcap_ends_it(built):
    """a truncated last record, an oversize record mid-capture (libpcap stops there), and a
    len > 262144 or zero len / caplen record (safe_pcap_next's exit; the output keeps the
    records before it)"""
    recs = S.records(S.pcap_fixed(20_000, 80, seed=12))
    pcap = S.build_pcap(recs)
    _run(pcap[:-30], ["--fixcsum"])
    ts, tu, cl, ln, d = recs[12_345]
    over = S.build_pcap(recs[:12_345]) + struct.pack("<IIII", ts, tu, 300_000, 300_000) + d + \
        S.build_pcap(recs[12_346:])[24:]
    _run(over, ["--fixcsum"])
    err = S.build_pcap(recs[:9_999] + [(ts, tu, cl, 400_000, d)] + recs[10_000:])
    _run(err, ["--fixcsum"])
    # safe_pcap_next's exit (src/common/utils.c:147-156): caplen 0, len 0, or both
    for zc, zl in ((0, 0), (0, 80), (cl, 0)):
        _run(S.build_pcap(recs[:7_777] + [(ts, tu, zc, zl, d[:zc])] + recs[7_778:]), ["--fixcsum"])


def test_record_like_payloads_fall_back_or_match(built):
    """payloads full of valid-looking record headers: a lane's guess may land inside a
    packet; the checks either repair it in the window or send the batch back to the host
    walk -- the output is the oracle's whichever happens"""
    fake = b"".join(struct.pack("<IIII", 1, 2, 12, 12) + bytes(range(12)) for _ in range(50))
    recs = []
    for ts, tu, cl, ln, d in S.records(S.pcap_fixed(4_000, 1_442, seed=13)):
        d = bytearray(d)
        d[42:42 + len(fake)] = fake
        recs.append((ts, tu, cl, ln, bytes(d)))
    _run(S.build_pcap(recs), ["--seed=3", "--fixcsum"], expect_applied=None)


def test_big_endian_and_nanosecond_captures(built):
    recs = S.records(S.pcap_imix(20_000, seed=14))
    for magic in (0xA1B23C4D, 0xD4C3B2A1):
        sw = magic == 0xD4C3B2A1
        e = ">" if sw else "<"
        hdr = struct.pack(e + "IHHiIII", 0xA1B2C3D4 if sw else magic, 2, 4, 0, 0, 65535, 1)
        body = b"".join(struct.pack(e + "IIII", ts, tu * (1000 if magic == 0xA1B23C4D else 1), cl, ln) + d
                        for ts, tu, cl, ln, d in recs)
        _run(hdr + body, ["--seed=5", "--fixcsum"])


def test_generic_configs_are_not_served(built):
    """a config whose tiles are the generic kernel's slots keeps the host index"""
    _run(S.pcap_imix(5_000, seed=15), ["--fixlen=pad", "--fixcsum"], expect_applied=False)


# ---------------------------------------------------------------- the pipeline's index
def _pipe(pcap, args, cache=None, chunk=1 << 20, env=None):
    import os
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        rc_o, exp = O.rewrite(pcap, args, cache)
        te = TA.TcpEdit(args)
        try:
            rc, out = te.rewrite_pipelined(pcap, cache, chunk_bytes=chunk)
        finally:
            te.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert rc == rc_o
    assert out == exp, f"first difference at byte {next(i for i in range(min(len(out), len(exp))) if out[i] != exp[i])}"


@pytest.mark.parametrize("name,gen,args", [
    ("c2", lambda: S.pcap_fixed(60_000, 64, seed=21), ["--seed=42", "--fixcsum"]),
    ("imix", lambda: S.pcap_imix(20_000, seed=22), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353",
                                                    "--fixcsum"]),
    ("c5", lambda: S.pcap_mixed_v4v6(4_000, 1514, seed=23), ["--fixcsum"]),
    ("efcs", lambda: S.pcap_imix(20_000, seed=24, fcs=True), ["--efcs", "--ttl=3"]),
    ("mixed", lambda: F.build(F.mixed(8000, seed=25)), ["--seed=7", "--fixcsum"]),
], ids=lambda x: x if isinstance(x, str) else "")
def test_pipeline_device_index_matches_the_oracle(built, name, gen, args):
    """the pipelined path: fixed 1 MiB chunks (records straddle every cut; the next chunk
    starts where the previous chain ended, read on the device) -- in window mode (the
    wave lane finds each chunk's records itself) where the config is size-preserving, and
    with the device record index (TCPEDIT_HIP_PIPE_NO_WIN)"""
    pcap = gen()
    _pipe(pcap, args)
    _pipe(pcap, args, env={"TCPEDIT_HIP_PIPE_NO_WIN": "1"})


def test_pipeline_device_index_edges(built):
    """records larger than a wave tile and than a generic slot across chunk cuts, caplen-0
    records, an oversize record (libpcap stops) and a len error in a later chunk, record-like
    payloads that fool the speculation (the chunk falls back to the host walk)"""
    base = S.records(S.pcap_fixed(30_000, 90, seed=26))
    big = S.records(S.pcap_fixed(3, 9000, seed=27)) + S.records(S.pcap_fixed(2, 200_000, seed=28))
    recs = []
    for i, r in enumerate(base):
        recs.append(r)
        if i % 97 == 0:
            recs.append((1, i, 1 + i % 21, 1 + i % 21, bytes(1 + i % 21)))
        if i % 89 == 5:
            ts, tu, cl, ln, d = r
            recs.append((ts, tu, cl, cl - 1 - i % 40, d))
        if i % 3001 == 0:
            recs.append(big[(i // 3001) % len(big)])
    args = ["--seed=3", "--fixcsum"]
    _pipe(S.build_pcap(recs), args)
    ts, tu, cl, ln, d = recs[25_000]
    over = S.build_pcap(recs[:25_000]) + struct.pack("<IIII", ts, tu, 300_000, 300_000) + d + \
        S.build_pcap(recs[25_001:])[24:]
    _pipe(over, args)
    err = S.build_pcap(recs[:22_222] + [(ts, tu, cl, 400_000, d)] + recs[22_223:])
    _pipe(err, args)
    fake = b"".join(struct.pack("<IIII", 1, 2, 12, 12) + bytes(range(12)) for _ in range(50))
    fooled = []
    for ts, tu, cl, ln, d in S.records(S.pcap_fixed(2_000, 1_442, seed=29)):
        d = bytearray(d)
        d[42:42 + len(fake)] = fake
        fooled.append((ts, tu, cl, ln, bytes(d)))
    _pipe(S.build_pcap(fooled), args)
    # the host walk in the pipeline (A/B) and the device index without the window mode:
    # the same bytes
    _pipe(S.build_pcap(recs), args, env={"TCPEDIT_HIP_PIPE_INDEX": "host"})
    _pipe(S.build_pcap(recs), args, env={"TCPEDIT_HIP_PIPE_NO_WIN": "1"})
    _pipe(over, args, env={"TCPEDIT_HIP_PIPE_NO_WIN": "1"})


def test_window_pipeline_chunk_cuts(built):
    """the window-mode pipeline over 1 MiB chunks: 64-byte records (the last record of
    every chunk straddles its cut, te_win_head completes the next image), 1,514-byte
    records, a capture one chunk long, and a capture whose last record is cut short (the
    chain ends early: the exact pipeline redoes the capture)"""
    args = ["--seed=42", "--fixcsum"]
    for pcap in (S.pcap_fixed(40_000, 64, seed=41), S.pcap_mixed_v4v6(3_000, 1514, seed=42),
                 S.pcap_fixed(5_000, 64, seed=43)):
        _pipe(pcap, args)
        _pipe(pcap[:-7], args)
