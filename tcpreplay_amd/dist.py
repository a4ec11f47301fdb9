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
        """shard k as a stand-alone pcap image (the input's file header + its records): a
        copy, for classifiers that take whole images; the rewrite path uses segment()"""
        return bytes(pcap[:PCAP_HDR_LEN]) + bytes(pcap[self.offsets[k]:self.offsets[k + 1]])

    def segment(self, pcap, k: int) -> memoryview:
        """shard k's records where they lie in `pcap` (bytes, bytearray or an mmap): no copy"""
        return memoryview(pcap)[self.offsets[k]:self.offsets[k + 1]]

    def count(self, k: int) -> int:
        nxt = self.pkt_base[k + 1] if k + 1 < len(self.pkt_base) else self.total
        return nxt - self.pkt_base[k]


@dataclass
class ShardResult:
    rc: int                   # TCPEDIT_OK / TCPEDIT_ERROR
    image: bytes              # output pcap image of the shard (header included)
    counters: List[int] = field(default_factory=lambda: [0] * len(COUNTER_NAMES))
    error: str = ""


def plan(pcap, n: int) -> ShardPlan:
    """tcpedit_pcap_shards (native host code) over an image in memory or an mmap of the
    file (read in place)."""
    from . import load, _buf
    L = load()
    f = L.tcpedit_pcap_shards
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                  ctypes.POINTER(ctypes.c_uint64)]
    off = (ctypes.c_uint64 * (n + 1))()
    base = (ctypes.c_uint64 * n)()
    keep, ptr, ln = _buf(pcap)
    total = f(ptr, ln, n, off, base)
    del keep
    if total < 0:
        raise ValueError("not a pcap image")
    return ShardPlan(list(off), list(base), int(total))


def fuzz_enabled(args) -> bool:
    """--fuzz-seed given: the one option whose records are not independent (fuzzing.c:87)"""
    return any(a == "--fuzz-seed" or a.startswith("--fuzz-seed=") for a in args)


def gpu_editor(image, args, cache: Optional[bytes], pkt_base: int, device: int,
               fuzz_prefix: Optional[Callable[[int], int]] = None, hdr=None) -> ShardResult:
    """Edit one shard on `device` through the C-ABI batch API.  `image` is a whole pcap
    image, or with `hdr` (the file header) the shard's records in place.  With
    --fuzz-seed, `fuzz_prefix(reaching records of this shard)` returns the RNG draws of
    every earlier shard, and the context's state skips them before the edit."""
    from . import Batch, TcpEdit
    te = TcpEdit(args, device=device)
    try:
        b = Batch(te, image, cache, pkt_base=pkt_base, hdr=hdr)
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
    if editor is None:  # the shard's records in place: no host copy
        dev = device if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
        res = gpu_editor(p.segment(pcap, rank), args, cache, p.pkt_base[rank], dev, fuzz_prefix=fz,
                         hdr=bytes(pcap[:PCAP_HDR_LEN]))
    elif fz is not None:
        res = editor(p.image(pcap, rank), args, cache, p.pkt_base[rank], fuzz_prefix=fz)
    else:
        res = editor(p.image(pcap, rank), args, cache, p.pkt_base[rank])
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


class _DeviceShard:
    """a rank's shard edited on its GPU, its output left in HBM until written"""

    def __init__(self, hdr, seg, args, cache, pkt_base, device, fuzz_prefix):
        from . import Batch, TcpEdit
        self.te = TcpEdit(args, device=device)
        self.b = None
        try:
            self.b = Batch(self.te, seg, cache, pkt_base=pkt_base, hdr=hdr)
            if fuzz_prefix is not None:
                self.te.fuzz_skip(fuzz_prefix(self.b.fuzz_reach()))
            self.rc = self.b.run()
            r = self.b.result()
        except Exception:
            self.close()
            raise
        self.counters = [int(getattr(r, n)) for n in COUNTER_NAMES]
        self.seg_len = max(0, int(r.out_len) - PCAP_HDR_LEN)
        self.error = self.te.geterr() if self.rc != 0 else ""

    def header(self) -> bytes:
        h = bytearray(PCAP_HDR_LEN)
        self.te._L.tcpedit_batch_output(self.b._b, (ctypes.c_char * PCAP_HDR_LEN).from_buffer(h), PCAP_HDR_LEN)
        return bytes(h)

    def write_into(self, view) -> int:
        return self.b.output_records_into(view)

    def close(self):
        if self.b is not None:
            self.b.close()
            self.b = None
        self.te.close()


class _HostShard:
    """a ShardResult from a caller's editor (the tests' oracle), written the same way"""

    def __init__(self, res: ShardResult):
        self.res, self.rc, self.counters, self.error = res, res.rc, res.counters, res.error
        self.seg_len = max(0, len(res.image) - PCAP_HDR_LEN)

    def header(self) -> bytes:
        return bytes(self.res.image[:PCAP_HDR_LEN])

    def write_into(self, view) -> int:
        n = min(len(view), self.seg_len)
        view[:n] = self.res.image[PCAP_HDR_LEN:PCAP_HDR_LEN + n]
        return n

    def close(self):
        pass


def rewrite_file_distributed(in_path: str, args, out_path: str, cache_path: Optional[str] = None,
                             device: Optional[int] = None, editor: Optional[Callable] = None):
    """tcprewrite -i in_path -o out_path [-c cache_path] over the ranks of an initialised
    torch.distributed group, sized for captures far larger than one host's share of RAM:

      * rank 0 plans the shards once over an mmap of the file (tcpedit_pcap_shards) and
        broadcasts the cut points (n+1 offsets, n record bases, the record count);
      * every rank mmaps the file and hands only its byte range, in place, to the device
        (tcpedit_batch_open_segment) -- no rank reads or copies another rank's records;
      * the ranks all-gather (segment bytes, error flag), rank 0 sizes the output file,
        and every rank D2H-copies its output records straight into an mmap of its range
        of that file (tcpedit_batch_output_records);
      * one all-reduce of the counters.

    Semantics are rewrite_distributed's (the first hard error in file order truncates the
    job's output).  --fuzz-seed adds its one exchange of reach counts.  `editor(hdr,
    records, cache, pkt_base[, fuzz_prefix]) -> ShardResult` replaces the device (CPU
    tests).  Returns (rc, counters dict, the output bytes this rank wrote, their offset)."""
    import mmap
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    cdev = _collective_device(dist)
    with open(in_path, "rb") as f:
        size = os.fstat(f.fileno()).st_size
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) if size else b""
    try:
        box = [None]
        if rank == 0:
            try:
                p = plan(mm, world)
                box = [(p.offsets, p.pkt_base, p.total, "")]
            except Exception as e:  # noqa: BLE001 -- every rank raises it below
                box = [(None, None, 0, str(e))]
        dist.broadcast_object_list(box, src=0)
        offsets, bases, total, perr = box[0]
        if perr:
            raise ValueError(perr)
        p = ShardPlan(offsets, bases, total)
        cache = None
        if cache_path is not None:
            with open(cache_path, "rb") as f:
                cache = f.read()  # header + n/4 bytes: the whole job's directions

        fz = None
        if fuzz_enabled(args):
            def fz(reach: int) -> int:
                mine = torch.tensor([reach], dtype=torch.int64, device=cdev)
                allv = [torch.zeros_like(mine) for _ in range(world)]
                dist.all_gather(allv, mine)
                return sum(int(v.item()) for v in allv[:rank])

        hdr = bytes(mm[:PCAP_HDR_LEN])
        sh, err = None, ""
        try:
            if editor is None:
                dev = device if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
                sh = _DeviceShard(hdr, p.segment(mm, rank), args, cache, p.pkt_base[rank], dev, fz)
            elif fz is not None:
                sh = _HostShard(editor(hdr, p.segment(mm, rank), cache, p.pkt_base[rank], fuzz_prefix=fz))
            else:
                sh = _HostShard(editor(hdr, p.segment(mm, rank), cache, p.pkt_base[rank]))
        except Exception as e:  # noqa: BLE001 -- travels in the all-gather below
            err = f"rank {rank}: {e}"
        try:
            # placement: (segment bytes, flag) from every rank; flag 1 a hard error in the
            # shard (tcprewrite.c:156-160), 2 the rank could not edit at all
            flag = 2 if sh is None else (0 if sh.rc == 0 else 1)
            mine = torch.tensor([0 if sh is None else sh.seg_len, flag], dtype=torch.int64, device=cdev)
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
            sizes = [int(v[0].item()) for v in allv]
            flags = [int(v[1].item()) for v in allv]
            if 2 in flags:
                raise RuntimeError(err or f"rank {flags.index(2)} failed to edit its shard")
            first_err = next((r_ for r_ in range(world) if flags[r_]), world)
            end = PCAP_HDR_LEN + sum(sizes[:first_err + 1 if first_err < world else world])
            offset = PCAP_HDR_LEN + sum(sizes[:rank]) if rank <= first_err else None
            write = sizes[rank] if rank <= first_err else 0

            cnt = torch.tensor(sh.counters, dtype=torch.int64, device=cdev)
            dist.all_reduce(cnt)
            job = dict(zip(COUNTER_NAMES, [int(x) for x in cnt.tolist()]))

            if rank == 0:  # tcprewrite's pcap_open_dead header, the file sized to the job
                with open(out_path, "wb") as f:
                    f.write(sh.header())
                    f.truncate(end)
            dist.barrier()
            if write:
                gran = mmap.ALLOCATIONGRANULARITY
                base = offset - offset % gran
                with open(out_path, "r+b") as f:
                    om = mmap.mmap(f.fileno(), offset - base + write, offset=base)
                    try:
                        got = sh.write_into(memoryview(om)[offset - base:offset - base + write])
                        om.flush()
                    finally:
                        om.close()
                if got != write:
                    raise RuntimeError(f"rank {rank}: wrote {got} of {write} output bytes")
            dist.barrier()
            return (-1 if first_err < world else 0), job, write, offset
        finally:
            if sh is not None:
                sh.close()
    finally:
        if isinstance(mm, mmap.mmap):
            mm.close()
