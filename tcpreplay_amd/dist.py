"""Multi-GPU tcprewrite: one process per GPU, packets sharded by byte-balanced
contiguous record ranges.

Records are independent for every en10mb->en10mb edit in scope, so a shard is
edited start to finish on its own GPU.  The only cross-rank traffic is
  * one all-gather of (output segment bytes, error flag) per rank -- 16 B each --
    from which every rank places its segment in the output file, and
  * one all-reduce (sum) of the counter vector: RCCL over xGMI when the process
    group is "nccl", gloo on CPU.
Each rank writes its own segment into the output file with pwrite; no packet
data crosses a collective.  --fuzz-seed adds one exchange before the edit: its RNG
is a single run-wide stream (fuzzing.c:8-20,87), so the ranks all-gather how many
of their records reach the fuzz step and each skips the draws of the ranks before it.

Hard errors keep tcprewrite's semantics (tcprewrite.c:156-160): the output is
cut at the first failing record in file order, so the first erroring shard is
truncated there and every later shard writes nothing.
"""
import ctypes
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional

COUNTER_NAMES = ("packets", "bytes_in", "bytes_out", "written", "edited", "soft_errors", "warnings", "errors",
                 "unsupported")
PCAP_HDR_LEN = 24


@dataclass
class ShardPlan:
    offsets: List[int]   # n+1 record-boundary byte offsets into the image
    pkt_base: List[int]  # global 0-based number of each shard's first record
    total: int           # records libpcap would read

    def image(self, pcap: bytes, k: int) -> bytes:
        """shard k as a stand-alone pcap image (the input's file header + its records)"""
        return bytes(pcap[:PCAP_HDR_LEN]) + bytes(pcap[self.offsets[k]:self.offsets[k + 1]])

    def count(self, k: int) -> int:
        nxt = self.pkt_base[k + 1] if k + 1 < len(self.pkt_base) else self.total
        return nxt - self.pkt_base[k]


@dataclass
class ShardResult:
    rc: int                   # TCPEDIT_OK / TCPEDIT_ERROR
    image: bytes              # output pcap image of the shard (header included)
    counters: List[int] = field(default_factory=lambda: [0] * len(COUNTER_NAMES))
    error: str = ""


def plan(pcap: bytes, n: int) -> ShardPlan:
    """tcpedit_pcap_shards (native host code) over an in-memory image."""
    from . import load
    L = load()
    f = L.tcpedit_pcap_shards
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                  ctypes.POINTER(ctypes.c_uint64)]
    off = (ctypes.c_uint64 * (n + 1))()
    base = (ctypes.c_uint64 * n)()
    total = f(pcap, len(pcap), n, off, base)
    if total < 0:
        raise ValueError("not a pcap image")
    return ShardPlan(list(off), list(base), int(total))


def fuzz_enabled(args) -> bool:
    """--fuzz-seed given: the one option whose records are not independent (fuzzing.c:87)"""
    return any(a == "--fuzz-seed" or a.startswith("--fuzz-seed=") for a in args)


def gpu_editor(image: bytes, args, cache: Optional[bytes], pkt_base: int, device: int,
               fuzz_prefix: Optional[Callable[[int], int]] = None) -> ShardResult:
    """Edit one shard on `device` through the C-ABI batch API.  With --fuzz-seed,
    `fuzz_prefix(reaching records of this shard)` returns the RNG draws of every earlier
    shard, and the context's state skips them before the edit."""
    from . import Batch, TcpEdit
    te = TcpEdit(args, device=device)
    try:
        b = Batch(te, image, cache, pkt_base=pkt_base)
        try:
            if fuzz_prefix is not None:
                te.fuzz_skip(fuzz_prefix(b.fuzz_reach()))
            rc = b.run()
            r = b.result()
            return ShardResult(rc, b.output(), [int(getattr(r, n)) for n in COUNTER_NAMES],
                               te.geterr() if rc != 0 else "")
        finally:
            b.close()
    finally:
        te.close()


def _collective_device(dist):
    import torch
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def rewrite_distributed(pcap: bytes, args, cache: Optional[bytes] = None, out_path: Optional[str] = None,
                        editor: Optional[Callable] = None, device: Optional[int] = None):
    """Run on every rank of an initialised torch.distributed group.

    Returns (rc, counters dict, segment bytes this rank wrote, its file offset).
    With `out_path` the ranks write the merged output file together.
    """
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    p = plan(pcap, world)
    shard = p.image(pcap, rank)
    cdev = _collective_device(dist)

    def fuzz_prefix(reach: int) -> int:
        # --fuzz-seed's one exchange: an exclusive prefix over ranks of the records that
        # reach the fuzz step (8 B per rank), so every shard's RNG stream starts where
        # the single-process run's would
        mine = torch.tensor([reach], dtype=torch.int64, device=cdev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        return sum(int(v.item()) for v in allv[:rank])

    fz = fuzz_prefix if fuzz_enabled(args) else None
    if editor is None:
        dev = device if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
        res = gpu_editor(shard, args, cache, p.pkt_base[rank], dev, fuzz_prefix=fz)
    elif fz is not None:
        res = editor(shard, args, cache, p.pkt_base[rank], fuzz_prefix=fz)
    else:
        res = editor(shard, args, cache, p.pkt_base[rank])
    seg = res.image[PCAP_HDR_LEN:]

    # 1) placement: (segment bytes, error flag) from every rank
    mine = torch.tensor([len(seg), 1 if res.rc < 0 else 0], dtype=torch.int64, device=cdev)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    sizes = [int(v[0].item()) for v in allv]
    errs = [int(v[1].item()) for v in allv]
    first_err = next((r for r in range(world) if errs[r]), world)
    if rank > first_err:
        seg = b""  # records after the first hard error are never written
    offset = PCAP_HDR_LEN + sum(sizes[:rank]) if rank <= first_err else None

    # 2) the job's counters: one all-reduce
    cnt = torch.tensor(res.counters, dtype=torch.int64, device=cdev)
    dist.all_reduce(cnt)
    counters = dict(zip(COUNTER_NAMES, [int(x) for x in cnt.tolist()]))

    if out_path is not None:
        end = PCAP_HDR_LEN + sum(sizes[:first_err + 1 if first_err < world else world])
        if rank == 0:
            with open(out_path, "wb") as f:
                f.write(res.image[:PCAP_HDR_LEN])
                f.truncate(end)
        dist.barrier()
        if seg:
            fd = os.open(out_path, os.O_WRONLY)
            try:
                os.pwrite(fd, seg, offset)
            finally:
                os.close(fd)
        dist.barrier()
    rc = -1 if first_err < world else 0
    return rc, counters, seg, offset
