"""Multi-GPU tcprewrite: one process per GPU, packets sharded by byte-balanced
contiguous record ranges.

Records are independent for every en10mb->en10mb edit in scope, so a shard is
edited start to finish on its own GPU.  The only cross-rank traffic is
  * one all-gather of (output segment bytes, error flag) per rank -- 16 B each --
    from which every rank places its segment in the output file, and
  * one all-reduce (sum) of the counter vector: RCCL over xGMI when the process
    group is "nccl", gloo on CPU.
Each rank writes its own segment into the output file with pwrite; no packet
data crosses a collective.  Before the edit the ranks exchange 24 B each -- (shard
opened, records reaching the fuzz step, dst_modified carry-out) -- for the two edits
that carry state across records: --fuzz-seed's RNG is a single run-wide stream
(fuzzing.c:8-20,87), so each rank skips the draws of the ranks before it; and a cooked,
Juniper or 802.11 decoder into en10mb without --enet-dmac carries the encoder's
dst_modified from the last C2S record to later ones (en10mb.c:597,612-615),
so each rank seeds its context with the nearest earlier shard's value.  Every rank
takes part in every collective even when its shard failed to open (it sends a sentinel
and all ranks raise after), so no rank is left waiting.

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


def place(sizes: List[int], errs: List[int]):
    """tcpedit_shard_place (native host code): where each shard's output records go in the
    job's file with tcprewrite's hard-error rule (tcprewrite.c:156-160) -- returns
    (offsets, bytes each shard writes, the file's size)"""
    from . import load
    L = load()
    f = L.tcpedit_shard_place
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int),
                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    n = len(sizes)
    off, wr = (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)()
    end = f(n, (ctypes.c_uint64 * n)(*sizes), (ctypes.c_int * n)(*[1 if e else 0 for e in errs]), off, wr)
    return list(off), list(wr), int(end)


def capture_dlt(hdr) -> int:
    """the DLT tcprewrite hands tcpedit_init (pcap_datalink of the file, tcprewrite.c:80):
    the header's link type in the file's byte order, LINKTYPE_RAW (101) as DLT_RAW (12)"""
    import struct
    h = bytes(hdr[:PCAP_HDR_LEN])
    if len(h) < PCAP_HDR_LEN:
        return 1
    big = h[:4] in (b"\xa1\xb2\xc3\xd4", b"\xa1\xb2\x3c\x4d")
    lt = struct.unpack_from(">I" if big else "<I", h, 20)[0] & 0x03FFFFFF
    return 12 if lt == 101 else lt


def fuzz_enabled(args) -> bool:
    """--fuzz-seed given: the one option whose records are not independent (fuzzing.c:87)"""
    return any(a == "--fuzz-seed" or a.startswith("--fuzz-seed=") for a in args)


def gpu_editor(image, args, cache: Optional[bytes], pkt_base: int, device: int,
               fuzz_prefix: Optional[Callable[[int], int]] = None, hdr=None) -> ShardResult:
    """Edit one shard on `device` through the C-ABI batch API (a single process: no
    exchange).  `image` is a whole pcap image, or with `hdr` (the file header) the shard's
    records in place.  With --fuzz-seed, `fuzz_prefix(reaching records of this shard)`
    returns the RNG draws of every earlier shard, and the context's state skips them."""
    sh = _DeviceShard(hdr, image, args, cache, pkt_base, device)
    try:
        sh.run(fuzz_prefix(sh.reach) if fuzz_prefix is not None else 0, None)
        return ShardResult(sh.rc, sh.b.output(), sh.counters, sh.error)
    finally:
        sh.close()


def _pre_edit(dist, cdev, sh):
    """The exchange before the edit, on every rank: (shard opened, fuzz reach,
    dst_modified carry-out) per rank -- for a Juniper capture the shards' decoder states
    first, then the carry-outs they decide (a second all-gather).  `sh`: this rank's
    _DeviceShard or None (it failed to open).  Returns (ranks that failed, fuzz draws of the
    earlier ranks, the dst_modified value the nearest earlier writing shard left, or 0: the
    reference's zeroed en10mb extra)."""
    import struct
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    ok = sh is not None
    jnpr = bool(ok and sh.jnpr)
    jv, jst = sh.jstate if ok else (False, bytes(48))
    words = list(struct.unpack("<6q", bytes(jst)[:48]))
    mine = torch.tensor([1 if ok else 0, sh.reach if ok else 0, sh.carry if ok else 2, 1 if jnpr else 0,
                         1 if jv else 0] + words, dtype=torch.int64, device=cdev)
    # (--fuzz-seed with the dst_modified carry: a fuzzed record's second encode writes it, so
    # a shard that fuzzes after earlier shards' draws finds its carry-out again from there)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    rows = [[int(x) for x in v.tolist()] for v in allv]
    bad = [r for r in range(world) if not rows[r][0]]
    skip = sum(rows[r][1] for r in range(rank))
    any_j = any(rows[r][3] for r in range(world))
    any_fz = any(rows[r][1] for r in range(world))
    if not bad and (any_j or any_fz):
        err = ""
        try:
            if any_j:  # the nearest earlier shard with a whole Juniper decode seeds this one's state
                src = next((r for r in range(rank - 1, -1, -1) if rows[r][4]), None)
                sh.seed_jnpr(struct.pack("<6q", *rows[src][5:11]) if src is not None else None)
            if any_fz:
                sh.skip_fuzz(skip)
        except Exception as e:  # noqa: BLE001 -- every rank raises after the exchange
            err = str(e)
        mine = torch.tensor([0 if err else 1, sh.carry if not err else 2], dtype=torch.int64, device=cdev)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        for r in range(world):
            rows[r][2] = int(allc[r][1].item())
            if not int(allc[r][0].item()):
                bad.append(r)
    carry_in = next((rows[r][2] for r in range(rank - 1, -1, -1) if rows[r][2] in (0, 1)), 0)
    return bad, skip, carry_in

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

    if editor is None:  # the shard's records in place: no host copy
        dev = device if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
        sh, err = None, ""
        try:
            sh = _DeviceShard(bytes(pcap[:PCAP_HDR_LEN]), p.segment(pcap, rank), args, cache, p.pkt_base[rank],
                              dev, prefix=memoryview(pcap)[PCAP_HDR_LEN:p.offsets[rank]] if rank else None)
        except Exception as e:  # noqa: BLE001 -- every rank raises after the exchange
            err = f"rank {rank}: {e}"
        bad, skip, carry_in = _pre_edit(dist, cdev, sh)
        if bad:
            if sh is not None:
                sh.close()
            raise RuntimeError(err or f"rank {bad[0]} failed to open its shard")
        try:
            sh.run(skip, carry_in)
            res = ShardResult(sh.rc, sh.b.output(), sh.counters, sh.error)
        finally:
            sh.close()
    elif fuzz_enabled(args):
        res = editor(p.image(pcap, rank), args, cache, p.pkt_base[rank], fuzz_prefix=fuzz_prefix)
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
    offs, writes, end = place(sizes, errs)
    if rank > first_err:
        seg = b""  # records after the first hard error are never written
    offset = offs[rank] if rank <= first_err else None

    # 2) the job's counters: one all-reduce
    cnt = torch.tensor(res.counters, dtype=torch.int64, device=cdev)
    dist.all_reduce(cnt)
    counters = dict(zip(COUNTER_NAMES, [int(x) for x in cnt.tolist()]))

    if out_path is not None:
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
    """a rank's shard on its GPU: opened (and its pre-edit facts found: records reaching
    the fuzz step, the dst_modified carry-out) by the constructor, edited by run(), its
    output left in HBM until written"""

    def __init__(self, hdr, seg, args, cache, pkt_base, device, prefix=None):
        from . import Batch, TcpEdit
        self.te = TcpEdit(args, dlt=capture_dlt(hdr if hdr is not None else seg), device=device)
        self.b, self.prefix = None, None
        self.fz_skipped = False
        try:
            self.b = Batch(self.te, seg, cache, pkt_base=pkt_base, hdr=hdr)
            if prefix is not None and len(prefix):
                # the earlier shards' records: read only if a record's edit reads the static
                # buffer past this shard's bytes, then the replay walks back into them
                self.prefix = prefix
                self.b.set_prefix(prefix)
            self.reach = self.b.fuzz_reach() if fuzz_enabled(args) else 0
            # DLT_JUNIPER_ETHER: the decoder state this shard's last whole inner decode
            # leaves goes round first; the dst_modified carry-out reads the seeded state
            # (a warning frame's destination is the carried one), so it waits for it
            self.jnpr = capture_dlt(hdr if hdr is not None else seg) == 178
            self.jstate = self.b.jnpr_out() if self.jnpr else (False, bytes(48))
            self.carry = 2 if self.jnpr else self.b.l2carry_out()
        except Exception:
            self.close()
            raise
        self.rc, self.counters, self.seg_len, self.error = None, [0] * len(COUNTER_NAMES), 0, ""

    def seed_jnpr(self, state):
        """the nearest earlier shard's Juniper decoder state (None: none before), then this
        shard's dst_modified carry-out, which reads it"""
        self.te.set_jnpr_state(state)
        self.carry = self.b.l2carry_out()

    def skip_fuzz(self, skip: int):
        """the earlier shards' fuzz draws (the RNG stream is run-wide); a shard that fuzzes
        after them finds its dst_modified carry-out again (a fuzzed record's second encode
        writes it)"""
        if skip:
            self.te.fuzz_skip(skip)
        self.fz_skipped = True
        if self.reach and skip:
            self.carry = self.b.l2carry_out()

    def run(self, fuzz_skip: int, carry_in: Optional[int]):
        """the edit, after the earlier shards' fuzz draws and with their carry"""
        if fuzz_skip and not self.fz_skipped:
            self.te.fuzz_skip(fuzz_skip)
        if carry_in is not None:
            self.te.set_l2carry(carry_in)
        self.rc = self.b.run()
        r = self.b.result()
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
        self.prefix = None  # (a view of the caller's mmap: released with the batch)
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
        if editor is None:
            dev = device if device is not None else int(os.environ.get("LOCAL_RANK", "0"))
            try:
                sh = _DeviceShard(hdr, p.segment(mm, rank), args, cache, p.pkt_base[rank], dev,
                                  prefix=memoryview(mm)[PCAP_HDR_LEN:p.offsets[rank]] if rank else None)
            except Exception as e:  # noqa: BLE001 -- travels in the exchange below
                err = f"rank {rank}: {e}"
            # every rank, opened or not: no rank is left waiting in a collective
            bad, skip, carry_in = _pre_edit(dist, cdev, sh)
            if sh is not None:
                try:
                    if bad:
                        raise RuntimeError(f"rank {bad[0]} failed to open its shard")
                    sh.run(skip, carry_in)
                except Exception as e:  # noqa: BLE001 -- travels in the all-gather below
                    err = err or f"rank {rank}: {e}"
                    sh.close()
                    sh = None
        else:
            try:
                if fz is not None:
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
            offs, writes, end = place(sizes, flags)
            offset = offs[rank] if rank <= first_err else None
            write = writes[rank]

            cnt = torch.tensor(sh.counters, dtype=torch.int64, device=cdev)
            dist.all_reduce(cnt)
            job = dict(zip(COUNTER_NAMES, [int(x) for x in cnt.tolist()]))

            if rank == 0:  # tcprewrite's pcap_open_dead header, the file sized to the job
                with open(out_path, "wb") as f:
                    f.write(sh.header())
                    f.truncate(end)
            dist.barrier()
            werr = ""
            if write:
                try:
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
                        werr = f"rank {rank}: wrote {got} of {write} output bytes"
                except Exception as e:  # noqa: BLE001 -- gathered below, raised on every rank
                    werr = f"rank {rank}: {e}"
            # the write outcome travels in a gather (not a barrier), so every rank raises
            okv = torch.tensor([0 if werr else 1], dtype=torch.int64, device=cdev)
            oks = [torch.zeros_like(okv) for _ in range(world)]
            dist.all_gather(oks, okv)
            if werr:
                raise RuntimeError(werr)
            failed = [r_ for r_ in range(world) if not int(oks[r_].item())]
            if failed:
                raise RuntimeError(f"rank {failed[0]} failed to write its output segment")
            return (-1 if first_err < world else 0), job, write, offset
        finally:
            if sh is not None:
                sh.close()
    finally:
        if isinstance(mm, mmap.mmap):
            mm.close()
