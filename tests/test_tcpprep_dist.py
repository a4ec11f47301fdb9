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


def _failing_table(rank_to_fail):
    def table(image, args, pkt_base):
        import torch.distributed as dist
        if dist.get_rank() == rank_to_fail:
            raise RuntimeError("no HIP device for the host-table pass")
        return _fake_table(image, args, pkt_base)
    return table


def _worker(rank, world, port, pcap, args, q, fail_rank=None, fake_auto=False):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        try:
            kw = {}
            if fail_rank is not None:
                kw["tabler"] = _failing_table(fail_rank)
            if fake_auto:
                kw = {"tabler": _fake_table, "comment": b""}
                q.put((rank, TP.prep_distributed(pcap, args, dist, classifier=_table_checking_classifier(pcap, world),
                                                 **kw)))
                return
            q.put((rank, TP.prep_distributed(pcap, args, dist, classifier=oracle_classifier, **kw)))
        except Exception as e:  # noqa: BLE001 -- the test checks every rank raised
            q.put((rank, f"raised: {type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def _run_world(pcap, args, world=2, fail_rank=None, fake_auto=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pcap, args, q, fail_rank, fake_auto))
             for r in range(world)]
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
    """the empty capture is refused on every rank before the collective, and a failure on
    one rank (here --auto's first pass on a box with no GPU) reaches every rank through the
    gathered tuple: nothing hangs in all_gather_object"""
    res = _run_world(synth.build_pcap([]), ["--port"])
    assert all(r.startswith("raised: ValueError") and "No packets" in r for r in res)
    res = _run_world(T.test_pcap(), ["--auto=bridge"], fail_rank=1)
    assert all(r.startswith("raised: RuntimeError") and "rank 1" in r for r in res)


def _fake_table(image, args, pkt_base):
    """a stand-in first pass (the real one needs the GPU): one node per record's index mod
    7, counted once per record, and the shard's base in a node of its own"""
    import numpy as np
    n = _records(image)
    keys = (1 << 63) | (np.arange(n, dtype=np.uint64) % np.uint64(7))
    keys = np.concatenate([keys, np.array([(1 << 62) + pkt_base], np.uint64)])
    return keys, np.ones(len(keys), np.uint64)


def _table_checking_classifier(full_pcap, world):
    def classify(image, args, pkt_base, merged=None):
        import numpy as np
        k, v = merged
        total = _records(full_pcap)
        assert len(k) == total + world and int(v.sum()) == total + world  # every rank's pairs, once
        assert sorted(int(x) for x in k if int(x) >> 62 == 1) == sorted(
            (1 << 62) + b for b in TP_plan_bases(full_pcap, world))
        return oracle_classifier(image, ["--port"], pkt_base)
    return classify


def TP_plan_bases(pcap, world):  # noqa: N802
    from tcpreplay_amd.dist import plan
    return plan(pcap, world).pkt_base


def test_auto_tables_are_exchanged_and_merged_on_every_rank(built):
    """gloo world_size 2: --auto's tables travel in one all_gather_object; every rank
    classifies with all of them (checked by the stand-in classifier)"""
    res = _run_world(T.test_pcap(), ["--auto=bridge"], fake_auto=True)
    exp = oracle_lib.tcpprep(T.test_pcap(), ["--no-arg-comment", "--port"])  # what the stand-in classifies by
    assert res[0] == res[1] == exp


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
def test_auto_shard_without_the_merged_table_is_refused():
    tp = TP.TcpPrep(["--auto=bridge"])
    tp.set_pkt_base(10)
    with pytest.raises(RuntimeError, match="auto_merge"):
        tp.cache(T.test_pcap())
    tp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bridge", "client", "server", "first", "router"])
def test_gpu_auto_shards_equal_unsharded(mode):
    """--auto over shards: each shard's host table, merged (counts add, the earliest
    sighting wins), then each shard classified by it -- the same cache as one pass over
    the whole capture, and as the oracle"""
    recs = synth.records(T.test_pcap())
    v6 = synth.records(synth.pcap_fixed(300, 90, ipv6=True, proto=6, seed=2))
    imix = synth.records(synth.pcap_imix(3000, seed=4))
    pcap = synth.build_pcap(recs + imix[:1500] + v6 + recs + imix[1500:])
    args = ["--no-arg-comment", "--auto=" + mode] + (["--ratio=0.5"] if mode == "client" else [])
    exp = oracle_lib.tcpprep(pcap, args)
    assert TP.cache(pcap, args) == exp
    assert TP.prep_distributed(pcap, args) == exp
