"""Python mirror of the gfx950 tcpprep classification pass (include/tcpprep.h).

Same option names as the reference's tcpprep (src/tcpprep_opts.def, long forms)
and the same output: a v04 cache file (src/common/cache.c:146-219).  The
classification runs in the kernel tp_classify of libtcpedit_hip.so; there is
no CPU path.
"""
import ctypes

from . import load as _load_lib

_SIG_DONE = False


def _lib():
    global _SIG_DONE
    L = _load_lib()
    if not _SIG_DONE:
        vp, c_int, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        for name, res, args in (
                ("tcpprep_init", c_int, [ctypes.POINTER(vp)]),
                ("tcpprep_parse_args", c_int, [vp, c_int, ctypes.POINTER(ctypes.c_char_p)]),
                ("tcpprep_cache_bound", sz, [vp, sz]),
                ("tcpprep_cache_pcap", ctypes.c_int64, [vp, ctypes.c_char_p, sz, vp, sz]),
                ("tcpprep_time", c_int, [vp, ctypes.c_char_p, sz, c_int, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_uint64)]),
                ("tcpprep_geterr", ctypes.c_char_p, [vp]),
                ("tcpprep_set_pkt_base", c_int, [vp, ctypes.c_uint64]),
                ("tcpprep_set_device", c_int, [vp, c_int]),
                ("tcpprep_last_entries", ctypes.c_int64, [vp]),
                ("tcpprep_auto_table", ctypes.c_int64, [vp, ctypes.c_char_p, sz, vp, vp, sz]),
                ("tcpprep_auto_merge", c_int, [vp, vp, vp, sz]),
                ("tcpprep_close", c_int, [ctypes.POINTER(vp)])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _SIG_DONE = True
    return L


class TcpPrep:
    """tcpprep_init + tcpprep_parse_args; cache(pcap) -> cache file bytes."""

    def __init__(self, args, device=None):
        self._L = _lib()
        self._ctx = ctypes.c_void_p()
        if self._L.tcpprep_init(ctypes.byref(self._ctx)) != 0:
            raise MemoryError("tcpprep_init failed")
        if device is not None and self._L.tcpprep_set_device(self._ctx, int(device)) != 0:
            self.close()
            raise ValueError(f"bad device {device}")
        argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
        if self._L.tcpprep_parse_args(self._ctx, len(args), argv) != 0:
            err = self.geterr()
            self.close()
            raise ValueError(err)

    def geterr(self):
        e = self._L.tcpprep_geterr(self._ctx)
        return e.decode() if e else ""

    def cache(self, pcap: bytes) -> bytes:
        cap = self._L.tcpprep_cache_bound(self._ctx, len(pcap))
        out = ctypes.create_string_buffer(cap)
        n = self._L.tcpprep_cache_pcap(self._ctx, pcap, len(pcap), out, cap)
        if n < 0:
            raise RuntimeError(self.geterr())
        return out.raw[:n]

    def set_pkt_base(self, base: int):
        if self._L.tcpprep_set_pkt_base(self._ctx, base) != 0:
            raise ValueError(self.geterr())

    def auto_table(self, pcap: bytes):
        """--auto over shards: this shard's host table -> (keys, values) uint64 arrays"""
        import numpy as np
        n = self._L.tcpprep_auto_table(self._ctx, pcap, len(pcap), None, None, 0)
        if n < 0:
            raise RuntimeError(self.geterr())
        k, v = np.zeros(max(n, 1), np.uint64), np.zeros(max(n, 1), np.uint64)
        m = self._L.tcpprep_auto_table(self._ctx, pcap, len(pcap), k.ctypes.data, v.ctypes.data, n)
        if m != n:
            raise RuntimeError(self.geterr() or "host table changed between calls")
        return k[:n], v[:n]

    def auto_merge(self, keys, vals):
        """every rank's (keys, values), concatenated: the table this shard classifies with"""
        import numpy as np
        k = np.ascontiguousarray(keys, np.uint64)
        v = np.ascontiguousarray(vals, np.uint64)
        if self._L.tcpprep_auto_merge(self._ctx, k.ctypes.data, v.ctypes.data, len(k)) != 0:
            raise RuntimeError(self.geterr())

    def last_entries(self) -> int:
        return self._L.tcpprep_last_entries(self._ctx)

    def time(self, pcap: bytes, iters=20):
        """(mean kernel ms, entries) with the image resident in HBM."""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        if self._L.tcpprep_time(self._ctx, pcap, len(pcap), iters, ctypes.byref(ms), ctypes.byref(n)) != 0:
            raise RuntimeError(self.geterr())
        return ms.value, n.value

    def close(self):
        if self._ctx:
            self._L.tcpprep_close(ctypes.byref(self._ctx))
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cache(pcap: bytes, args) -> bytes:
    tp = TcpPrep(args)
    try:
        return tp.cache(pcap)
    finally:
        tp.close()


def _local_rank():
    import os
    v = os.environ.get("LOCAL_RANK")
    return int(v) if v is not None else None


def gpu_classifier(image: bytes, args, pkt_base: int, device=None, merged=None):
    """one shard on the GPU (LOCAL_RANK's device by default, as gpu_editor) ->
    (cache body bytes, entries, the cache comment); merged: --auto's table from every rank"""
    tp = TcpPrep(args, device=_local_rank() if device is None else device)
    try:
        tp.set_pkt_base(pkt_base)
        if merged is not None:
            tp.auto_merge(*merged)
        c = tp.cache(image)
        clen = int.from_bytes(c[22:24], "big")
        return c[24 + clen:], tp.last_entries(), c[24:24 + clen]
    finally:
        tp.close()


def gpu_auto_table(image: bytes, args, pkt_base: int, device=None):
    """--auto over shards, first pass: one shard's host table on the GPU -> (keys, values)"""
    tp = TcpPrep(args, device=_local_rank() if device is None else device)
    try:
        tp.set_pkt_base(pkt_base)
        return tp.auto_table(image)
    finally:
        tp.close()


def merge_shards(parts, records: int, comment: bytes) -> bytes:
    """(body, entries[, comment]) per shard in file order -> one v04 cache file: the
    shards' 2-bit entries concatenated (a shard's entry count need not be a multiple of 4)."""
    import numpy as np
    ents = []
    for part in parts:
        body, n = part[0], part[1]
        b = np.frombuffer(body, np.uint8)
        e = ((b[:, None] >> np.array([0, 2, 4, 6], np.uint8)) & 3).reshape(-1)[:n]
        ents.append(e)
    e = np.concatenate(ents) if ents else np.zeros(0, np.uint8)
    pad = (-len(e)) % 4
    e = np.concatenate([e, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    body = (e[:, 0] | (e[:, 1] << 2) | (e[:, 2] << 4) | (e[:, 3] << 6)).astype(np.uint8).tobytes()
    hdr = b"tcpprep\0" + b"04\0\0" + records.to_bytes(8, "big") + (4).to_bytes(2, "big") + \
        len(comment).to_bytes(2, "big")
    return hdr + comment + body


def comment_of(args) -> bytes:
    """the cache comment the options give (read back from a one-record probe run; only
    for classifiers that do not return it)"""
    from . import synth
    tp = TcpPrep(args)
    try:
        c = tp.cache(synth.pcap_fixed(1, 64))
    finally:
        tp.close()
    return c[24:24 + int.from_bytes(c[22:24], "big")]


def _is_auto(args) -> bool:
    return any(a == "-a" or a.startswith("--auto") for a in args)


def _exchange(dist, world, fn):
    """fn() on this rank (or every shard with dist=None); one all_gather_object of
    (ok, result or error) per rank, and every rank raises the same error"""
    if dist:
        r = dist.get_rank()
        try:
            mine = (True, fn(r))
        except Exception as e:  # noqa: BLE001 -- reported on every rank below
            mine = (False, f"rank {r}: {e}")
        got = [None] * world
        dist.all_gather_object(got, mine)
        errs = [m[1] for m in got if not m[0]]
        if errs:
            raise RuntimeError("; ".join(errs))
        return [m[1] for m in got]
    return [fn(k) for k in range(world)]


def prep_distributed(pcap: bytes, args, dist=None, classifier=None, comment: bytes = None, tabler=None):
    """Sharded tcpprep: each rank classifies its byte-balanced record range
    (tcpedit_pcap_shards) with its global record base, one all_gather_object of
    (ok, (body, entries[, comment]) or error) per rank, every rank assembles the same
    cache file -- or every rank raises the same error.  With dist=None all shards run in
    this process (one per 'rank' of a 2-way plan).

    --auto first exchanges each shard's host table (tabler: the first pass, tree.c's
    nodes with their counts / first sightings at global record numbers); every rank
    merges all of them (tcpprep_auto_merge: counts add, the earliest sighting wins) and
    classifies its shard by the whole capture's table, as the reference's one pass does.

    Decisions that end the job are taken identically on every rank before the collective
    (an empty capture is the reference's "No packets were processed"), and a failure on one
    rank travels in the gathered tuple, so no rank is left waiting in a collective."""
    import numpy as np
    from .dist import plan
    classifier = classifier or gpu_classifier
    tabler = tabler or gpu_auto_table
    world = dist.get_world_size() if dist else 2
    p = plan(pcap, world)
    if p.total == 0:
        raise ValueError("No packets were processed.  Filter too limiting?")
    auto = world > 1 and _is_auto(args)
    merged = None
    if auto:
        def table(k):
            if p.count(k) == 0:
                return (np.zeros(0, np.uint64), np.zeros(0, np.uint64))
            return tabler(p.image(pcap, k), args, p.pkt_base[k])
        tabs = _exchange(dist, world, table)
        merged = (np.concatenate([t[0] for t in tabs]), np.concatenate([t[1] for t in tabs]))

    def run(k):
        if p.count(k) == 0:  # a shard holding only the file header (fewer records than ranks)
            return (b"", 0, None)
        if auto:
            return classifier(p.image(pcap, k), args, p.pkt_base[k], merged=merged)
        return classifier(p.image(pcap, k), args, p.pkt_base[k])

    parts = _exchange(dist, world, run)
    if comment is None:
        comment = next((pt[2] for pt in parts if len(pt) > 2 and pt[2] is not None), None)
    if comment is None:
        comment = comment_of(args)
    return merge_shards(parts, p.total, comment)
