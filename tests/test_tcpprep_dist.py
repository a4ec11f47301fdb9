"""Sharded tcpprep (tcpreplay_amd.tcpprep.prep_distributed): byte-balanced record
ranges per rank, one all_gather_object of (cache body, entries), shards' 2-bit
entries concatenated.  gloo world_size 2 on CPU with the oracle as the per-shard
classifier, and the GPU classifier in one process against the unsharded run."""
import multiprocessing as mp
import socket

import pytest

import oracle_lib
import tcpprep_cases as T
from tcpreplay_amd import synth
from tcpreplay_amd import tcpprep as TP


def _records(image: bytes) -> int:
    return len(synth.records(image))


def oracle_classifier(image, args, pkt_base):
    """the oracle on one shard, with global record numbers for P: lists and its own entry
    count (MAC mode gives short records no entry)"""
    c, n = oracle_lib.tcpprep(image, args, pkt_base=pkt_base, with_entries=True)
    clen = int.from_bytes(c[22:24], "big")
    return c[24 + clen:], n, c[24:24 + clen]


def _worker(rank, world, port, pcap, args, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        try:
            q.put((rank, TP.prep_distributed(pcap, args, dist, classifier=oracle_classifier)))
        except Exception as e:  # noqa: BLE001 -- the test checks every rank raised
            q.put((rank, f"raised: {type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def _run_world(pcap, args, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pcap, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return [r[1] for r in res]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_merge_places_entries_at_two_bit_granularity():
    parts = [(bytes([0b11100110]), 3), (bytes([0b10111110, 0b11]), 5)]
    c = TP.merge_shards(parts, 8, b"x")
    assert c[:24] == b"tcpprep\0" + b"04\0\0" + (8).to_bytes(8, "big") + b"\0\x04\0\x01"
    # entries 10,01,10 | 10,11,11,10,11 -> bytes 0b10_10_01_10, 0b11_10_11_11
    assert c[24:] == b"x" + bytes([0b10100110, 0b11101111])


def _mac_capture():
    """test.pcap with short records (no MAC-mode entry) on both sides of the split"""
    recs = synth.records(T.test_pcap())
    recs.insert(30, (0, 0, 10, 10, bytes(10)))
    recs.insert(150, (0, 0, 5, 5, bytes(5)))
    return synth.build_pcap(recs)


@pytest.mark.parametrize("args", [["--port"], ["--cidr=96.17.211.0/24", "--reverse"],
                                  ["--cidr=96.17.211.0/24", "--include=P:3-70,120-"],
                                  ["--port", "--exclude=P:91-100"],
                                  ["--mac=00:1f:f3:3c:e1:13", "--exclude=P:5"]])
def test_two_rank_prep_equals_single_process(built, args):
    """gloo world_size 2: global P: numbering and MAC-mode entry counts across shards"""
    pcap = _mac_capture() if any(a.startswith("--mac") for a in args) else T.test_pcap()
    res = _run_world(pcap, args)
    exp = oracle_lib.tcpprep(pcap, args)
    assert res[0] == exp and res[1] == exp


def test_fewer_records_than_ranks(built):
    """a 1-record capture at world 2: rank 1's shard holds only the file header and
    contributes no entries (no classifier call, no 'No packets were processed')"""
    pcap = synth.build_pcap(synth.records(T.test_pcap())[:1])
    args = ["--no-arg-comment", "--port"]
    res = _run_world(pcap, args)
    exp = oracle_lib.tcpprep(pcap, args)
    assert res[0] == exp and res[1] == exp


def test_every_rank_raises_together(built):
    """--auto and the empty capture are refused on every rank before the collective;
    nothing hangs in all_gather_object"""
    res = _run_world(T.test_pcap(), ["--auto=bridge"])
    assert all(r.startswith("raised: ValueError") for r in res)
    res = _run_world(synth.build_pcap([]), ["--port"])
    assert all(r.startswith("raised: ValueError") and "No packets" in r for r in res)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--port"], ["--cidr=10.0.0.0/9", "--include=P:3-700,900-"],
                                  ["--mac=00:1f:f3:3c:e1:13", "--exclude=P:5"]])
def test_gpu_shards_equal_unsharded(args):
    recs = synth.records(synth.pcap_imix(5001, seed=9)) + synth.records(T.test_pcap())
    recs.insert(2600, (0, 0, 10, 10, bytes(10)))  # MAC mode: a record with no entry, in shard 2
    pcap = synth.build_pcap(recs)
    args = ["--no-arg-comment"] + args
    assert TP.prep_distributed(pcap, args) == TP.cache(pcap, args) == oracle_lib.tcpprep(pcap, args)


@pytest.mark.gpu
def test_auto_modes_refuse_a_shard_base():
    tp = TP.TcpPrep(["--auto=bridge"])
    with pytest.raises(ValueError):
        tp.set_pkt_base(10)
    tp.close()
