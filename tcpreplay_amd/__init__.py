"""tcpreplay_amd -- MI355X-native tcpedit (tcprewrite's per-packet edit engine).

Python mirror of the reference's libtcpedit interface (src/tcpedit/tcpedit.h,
parse_args.h, tcpedit_api.h) over the C-ABI of the in-tree native library
tcpreplay_amd/lib/libtcpedit_hip.so.  Every packet edit runs in the gfx950
kernels; there is no Python or CPU edit path, and importing the native library
fails loudly when it has not been built.
"""
import ctypes
import struct
import os

__all__ = ["TcpEdit", "Batch", "BatchResult", "load", "LIB_PATH", "TCPEDIT_OK", "TCPEDIT_ERROR",
           "TCPEDIT_SOFT_ERROR", "TCPEDIT_WARN", "ST"]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TCPEDIT_HIP_LIB") or os.path.join(HERE, "lib", "libtcpedit_hip.so")

TCPEDIT_SOFT_ERROR, TCPEDIT_ERROR, TCPEDIT_OK, TCPEDIT_WARN = -2, -1, 0, 1
TCPR_DIR_NOSEND, TCPR_DIR_C2S, TCPR_DIR_S2C = 0, 1, 2
JNPR_STATE_BYTES = 48  # TCPEDIT_JNPR_STATE_BYTES


class ST:
    """per-record status bits (te_dev_cfg.h)"""
    RC_MASK, OK, WARN, SOFT, ERROR = 0x03, 0, 1, 2, 3
    DROPPED, NOSEND, UNSUPPORTED, WARNED, ZEROCAP = 0x04, 0x08, 0x10, 0x20, 0x40


class BatchResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("packets", "bytes_in", "bytes_out", "written", "edited", "soft_errors", "warnings", "errors",
                 "unsupported", "out_len")] + [
        ("first_error", ctypes.c_int64), ("first_unsupported", ctypes.c_int64), ("n_tiles", ctypes.c_uint32),
        ("kernel_ms", ctypes.c_double), ("fast_lane", ctypes.c_uint32), ("generic_tiles", ctypes.c_uint32),
        ("fast_kind", ctypes.c_uint32), ("stale_records", ctypes.c_uint64)]

FAST_KERNELS = {1: "te_fast_tiles", 2: "te_wave_tiles"}


class PcapPkthdr(ctypes.Structure):
    _fields_ = [("tv_sec", ctypes.c_long), ("tv_usec", ctypes.c_long), ("caplen", ctypes.c_uint32),
                ("len", ctypes.c_uint32)]


_lib = None


def load():
    """Load the native library (no fallback: a missing build is an error)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C tcpreplay_amd/csrc` "
                          "(or __graft_entry__.build()); tcpreplay_amd has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, c_int, u64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "tcpedit_init": (c_int, [ctypes.POINTER(vp), c_int]),
        "tcpedit_geterr": (ctypes.c_char_p, [vp]),
        "tcpedit_getwarn": (ctypes.c_char_p, [vp]),
        "tcpedit_checkerror": (c_int, [vp, c_int, ctypes.c_char_p]),
        "tcpedit_validate": (c_int, [vp]),
        "tcpedit_packet": (c_int, [vp, ctypes.POINTER(ctypes.POINTER(PcapPkthdr)),
                                   ctypes.POINTER(ctypes.c_char_p), c_int]),
        "tcpedit_close": (c_int, [ctypes.POINTER(vp)]),
        "tcpedit_get_output_dlt": (c_int, [vp]),
        "tcpedit_l3data": (vp, [vp, c_int, vp, c_int]),
        "tcpedit_l3proto": (c_int, [vp, c_int, vp, c_int]),
        "tcpedit_get_total_bytes": (u64, [vp]),
        "tcpedit_get_pkts_edited": (u64, [vp]),
        "tcpedit_post_args": (c_int, [vp]),
        "tcpedit_set_option": (c_int, [vp, ctypes.c_char_p, ctypes.c_char_p]),
        "tcpedit_parse_args": (c_int, [vp, c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_int)]),
        "tcpedit_batch_open": (vp, [vp, vp, sz, vp, sz, u64]),
        "tcpedit_batch_run": (c_int, [vp, vp]),
        "tcpedit_batch_run_fused": (c_int, [vp, vp]),
        "tcpedit_batch_time_fused": (c_int, [vp, vp, c_int, ctypes.POINTER(ctypes.c_double)]),
        "tcpedit_batch_fused_fallbacks": (ctypes.c_uint64, [vp]),
        "tcpedit_pipeline_fallbacks": (ctypes.c_uint64, [vp]),
        "tcpedit_batch_update_input": (c_int, [vp, vp, vp, sz]),
        "tcpedit_batch_set_prefix": (c_int, [vp, vp, vp, sz]),
        "tcpedit_batch_result": (c_int, [vp, ctypes.POINTER(BatchResult)]),
        "tcpedit_batch_output": (sz, [vp, vp, sz]),
        "tcpedit_batch_open_segment": (vp, [vp, vp, vp, sz, vp, sz, u64]),
        "tcpedit_batch_output_records": (sz, [vp, vp, sz]),
        "tcpedit_batch_status": (ctypes.POINTER(ctypes.c_uint8), [vp]),
        "tcpedit_batch_time": (c_int, [vp, vp, c_int, ctypes.POINTER(ctypes.c_double)]),
        "tcpedit_batch_time_kernels": (c_int, [vp, vp, c_int, ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_double)]),
        "tcpedit_batch_close": (None, [vp]),
        "tcpedit_batch_index_device": (c_int, [vp, vp, c_int, ctypes.POINTER(ctypes.c_double)]),
        "tcpedit_batch_fuzz_reach": (ctypes.c_int64, [vp, vp]),
        "tcpedit_fuzz_skip": (c_int, [vp, u64]),
        "tcpedit_batch_l2carry_out": (c_int, [vp, vp]),
        "tcpedit_set_l2carry": (c_int, [vp, c_int]),
        "tcpedit_batch_jnpr_out": (c_int, [vp, vp, vp, ctypes.c_size_t]),
        "tcpedit_set_jnpr_state": (c_int, [vp, vp, ctypes.c_size_t, c_int]),
        "tcpedit_batch_device_output": (vp, [vp]),
        "tcpedit_batch_input_bytes": (u64, [vp]),
        "tcpedit_rewrite_pcap": (c_int, [vp, vp, sz, vp, sz, ctypes.POINTER(vp), ctypes.POINTER(sz)]),
        "tcpedit_rewrite_pcap_pipelined": (c_int, [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(sz), sz]),
        "tcpedit_output_bound": (sz, [vp, vp, sz]),
        "tcpedit_host_alloc": (vp, [sz]),
        "tcpedit_host_free": (None, [vp]),
        "tcpedit_set_device": (c_int, [c_int]),
        "tcpedit_get_dev_cfg": (c_int, [vp, vp, sz, vp]),
        "tcpedit_replay_open": (vp, [vp, vp, sz, c_int]),
        "tcpedit_replay_bound": (sz, [vp, vp]),
        "tcpedit_replay_pass": (c_int, [vp, vp, vp, sz, ctypes.POINTER(sz)]),
        "tcpedit_replay_close": (None, [vp]),
        "tcpedit_replay_parse_args": (c_int, [vp, vp, c_int, ctypes.POINTER(ctypes.c_char_p)]),
        "tcpedit_replay_failed": (ctypes.c_uint64, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _lib = L
    return L


class PinnedBuffer:
    """Page-locked host memory from the library (tcpedit_host_alloc); `.view` is a
    writable memoryview of it.  A capture read into one crosses PCIe by DMA without the
    per-call page locking of an ordinary buffer."""

    def __init__(self, nbytes):
        self._L = load()
        self.nbytes = int(nbytes)
        self._p = self._L.tcpedit_host_alloc(max(1, self.nbytes))
        if not self._p:
            raise MemoryError(f"tcpedit_host_alloc({nbytes}) failed")
        self.view = memoryview((ctypes.c_char * self.nbytes).from_address(self._p)).cast("B")

    def close(self):
        if self._p:
            self.view.release()
            self._L.tcpedit_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _buf(data):
    """(keep-alive, address, length) of any bytes-like object (bytes, bytearray,
    memoryview, mmap, numpy array) without copying it; (None, None, 0) for None"""
    if data is None:
        return None, None, 0
    import numpy as np
    a = np.frombuffer(data, np.uint8)
    return a, a.ctypes.data, a.size


class TcpEdit:
    """A tcpedit context: tcpedit_init + option surface + tcpedit_post_args.

    `args` uses tcprewrite's tcpedit/DLT options, e.g. ["--seed=42", "--fixcsum"];
    "--skip-soft-errors" (a tcprewrite option) is accepted too.
    """

    def __init__(self, args=(), dlt=1, device=None):
        L = load()
        if device is not None:
            L.tcpedit_set_device(int(device))
        self._L = L
        self._ctx = ctypes.c_void_p()
        rc = L.tcpedit_init(ctypes.byref(self._ctx), dlt)
        if rc < 0:
            err = L.tcpedit_geterr(self._ctx).decode() if self._ctx else "init failed"
            raise RuntimeError(err)
        args = list(args)
        argv = (ctypes.c_char_p * max(1, len(args)))(*[a.encode() for a in args])
        unused = (ctypes.c_int * max(1, len(args)))()
        n = L.tcpedit_parse_args(self._ctx, len(args), argv, unused)
        if n < 0:
            raise ValueError(self.geterr())
        extra = [args[unused[i]] for i in range(n)]
        for a in extra:
            if a == "--skip-soft-errors":
                L.tcpedit_set_option(self._ctx, b"skip-soft-errors", None)
            else:
                raise ValueError(f"unknown option {a}")
        if L.tcpedit_post_args(self._ctx) < 0:
            raise ValueError(self.geterr())
        L.tcpedit_validate(self._ctx)

    def geterr(self):
        return self._L.tcpedit_geterr(self._ctx).decode(errors="replace")

    @property
    def pipeline_fallbacks(self) -> int:
        """pipelined calls whose window mode missed and that redid the capture the exact way
        (tcpedit_pipeline_fallbacks)"""
        return int(self._L.tcpedit_pipeline_fallbacks(self._ctx))

    def close(self):
        if self._ctx:
            self._L.tcpedit_close(ctypes.byref(self._ctx))
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rewrite(self, pcap: bytes, cache: bytes = None, with_status=False):
        """Whole-file rewrite (tcprewrite semantics).  Returns (rc, out_bytes[, status])."""
        b = Batch(self, pcap, cache)
        try:
            rc = b.run()
            out = b.output()
            if with_status:
                return rc, out, b.status()
            return rc, out
        finally:
            b.close()

    def output_bound(self, pcap):
        """worst-case output size of `pcap` under this context's options"""
        src = pcap if isinstance(pcap, (bytearray, memoryview)) else bytearray(pcap)
        return self._L.tcpedit_output_bound(self._ctx, (ctypes.c_char * len(src)).from_buffer(src), len(src))

    def rewrite_pipelined(self, pcap, cache: bytes = None, chunk_bytes=0, out=None):
        """Whole-file rewrite through the chunked H2D | edit | D2H pipeline.  `pcap` may be
        bytes or any writable buffer; `out` an optional preallocated bytearray (reused across
        calls).  Returns (rc, output as a memoryview of `out` or bytes)."""
        L = self._L
        src = pcap if isinstance(pcap, (bytearray, memoryview)) else bytearray(pcap)
        n = len(src)
        inp = (ctypes.c_char * n).from_buffer(src)
        own = out is None  # a caller's `out` is checked against the output by the library
        if own:
            out = bytearray(max(L.tcpedit_output_bound(self._ctx, inp, n), 24))
        ob = (ctypes.c_char * len(out)).from_buffer(out)
        _kc, cb, cn = _buf(cache)
        olen = ctypes.c_size_t(0)
        rc = L.tcpedit_rewrite_pcap_pipelined(self._ctx, inp, n, cb, cn, ob, len(out), ctypes.byref(olen),
                                              int(chunk_bytes))
        if own:
            return rc, bytes(memoryview(out)[:olen.value])
        return rc, memoryview(out)[:olen.value]

    def fuzz_skip(self, draws: int):
        """advance the --fuzz-seed state by `draws` tcpr_random() calls (tcpedit_fuzz_skip)"""
        if self._L.tcpedit_fuzz_skip(self._ctx, int(draws)) < 0:
            raise RuntimeError(self.geterr())

    def set_l2carry(self, value: int):
        """seed the en10mb encoder's dst_modified carry as an earlier shard
        left it (tcpedit_set_l2carry)"""
        if self._L.tcpedit_set_l2carry(self._ctx, int(value)) < 0:
            raise RuntimeError(self.geterr())

    def set_jnpr_state(self, state=None, unknown: bool = False):
        """seed the Juniper decoder state (the state a frame whose extensions are not Ethernet
        is encoded with, jnpr_ether.c:269-272) as an earlier shard left it (Batch.jnpr_out);
        None: the capture's start (tcpedit_set_jnpr_state)"""
        buf = ctypes.create_string_buffer(bytes(state), JNPR_STATE_BYTES) if state is not None else None
        if self._L.tcpedit_set_jnpr_state(self._ctx, buf, JNPR_STATE_BYTES, 1 if unknown else 0) < 0:
            raise RuntimeError(self.geterr())

    def packet(self, hdr, data: bytearray, direction=TCPR_DIR_C2S):
        """tcpedit_packet(): edits `data` (bytearray, >= MAXPACKET bytes recommended) in place.

        hdr = dict(ts_sec, ts_usec, caplen, len); returns (rc, new_hdr)."""
        h = PcapPkthdr(hdr.get("ts_sec", 0), hdr.get("ts_usec", 0), hdr["caplen"], hdr["len"])
        hp = ctypes.pointer(h)
        buf = (ctypes.c_char * len(data)).from_buffer(data)
        dp = ctypes.c_char_p(ctypes.addressof(buf))
        rc = self._L.tcpedit_packet(self._ctx, ctypes.byref(hp), ctypes.byref(dp), direction)
        return rc, {"ts_sec": h.tv_sec, "ts_usec": h.tv_usec, "caplen": h.caplen, "len": h.len}


class Replay:
    """tcpreplay-edit's send loop over one capture, batched (tcpedit_replay_open): each
    pass() edits every record as send_packets' tcpedit_packet call does
    (send_packets.c:469-474) and returns the records as sent, in the -w dump's form
    (16-byte headers with nanosecond fractions, no file header).  With preload (-K) the
    passes after the first edit the cached copy in place, so edits compound."""

    def __init__(self, te: TcpEdit, pcap, preload=False, replay_args=()):
        """replay_args: tcpreplay's own options on this path (--include=LIST, --exclude=LIST,
        --unique-ip, --unique-ip-loops=N; tcpedit_replay_parse_args)"""
        self._te, self._L = te, te._L
        keep, p, n = _buf(pcap)
        self._r = self._L.tcpedit_replay_open(te._ctx, p, n, 1 if preload else 0)
        del keep
        if not self._r:
            raise RuntimeError(te.geterr())
        if replay_args:
            argv = (ctypes.c_char_p * len(replay_args))(*[a.encode() for a in replay_args])
            if self._L.tcpedit_replay_parse_args(te._ctx, self._r, len(replay_args), argv) != 0:
                err = te.geterr()
                self.close()
                raise ValueError(err)
        self._cap = self._L.tcpedit_replay_bound(te._ctx, self._r)

    @property
    def failed(self):
        """records whose --unique-ip edit failed so far (not sent)"""
        return int(self._L.tcpedit_replay_failed(self._r))

    def pass_(self):
        """one --loop pass: (rc, records as sent); rc < 0 ends the run (errx), the
        records before the failing one still returned"""
        out = ctypes.create_string_buffer(max(1, self._cap))
        n = ctypes.c_size_t(0)
        rc = self._L.tcpedit_replay_pass(self._te._ctx, self._r, out, self._cap, ctypes.byref(n))
        return rc, out.raw[:n.value]

    def close(self):
        if self._r:
            self._L.tcpedit_replay_close(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# pcap_open_dead(DLT_EN10MB, MAX_SNAPLEN) + pcap_dump_open (sendpacket.c:945-968)
REPLAY_DUMP_HEADER = struct.pack("<IHHiIII", 0xa1b2c3d4, 2, 4, 0, 0, 262144, 1)


REPLAY_OPTS = ("--include=", "--exclude=", "--unique-ip-loops=")


def split_replay_args(args):
    """tcpreplay's own options on the tcpreplay-edit path, and the tcpedit options"""
    mine = [a for a in args if a == "--unique-ip" or a.startswith(REPLAY_OPTS)]
    return mine, [a for a in args if a not in mine]


def replay_edit(pcap, args, loops=1, preload=False, errors=None):
    """`tcpreplay-edit -w out --loop=loops [-K] <args> in.pcap`: (rc, the -w file's bytes);
    a failing pass's error string is appended to `errors` (a list) when given"""
    rargs, eargs = split_replay_args(args)
    te = TcpEdit(eargs)
    try:
        r = Replay(te, pcap, preload, rargs)
        try:
            out, rc = [REPLAY_DUMP_HEADER], 0
            for p in range(int(loops)):
                rc, recs = r.pass_()
                out.append(recs)
                if rc < 0:
                    if errors is not None:
                        errors.append(f"pass {p}: {te.geterr()}")
                    break
            return rc, b"".join(out)
        finally:
            r.close()
    finally:
        te.close()


class Batch:
    """A pcap image staged in HBM (tcpedit_batch_open).  With `hdr` (the file's 24-byte
    header), `pcap` is a segment of whole records -- e.g. a rank's byte range of an mmap'd
    capture -- read in place (tcpedit_batch_open_segment).  No host copy is made of
    either: any bytes-like object is passed by address."""

    def __init__(self, te: TcpEdit, pcap, cache=None, pkt_base=0, hdr=None):
        self._te, self._L = te, te._L
        keep, p, n = _buf(pcap)
        kc, c, cn = _buf(cache)
        if hdr is None:
            self._b = self._L.tcpedit_batch_open(te._ctx, p, n, c, cn, pkt_base)
        else:
            kh, h, hn = _buf(hdr)
            if hn < 24:
                raise ValueError("hdr: the 24-byte pcap file header")
            self._b = self._L.tcpedit_batch_open_segment(te._ctx, h, p, n, c, cn, pkt_base)
        del keep, kc  # the library has read and uploaded both
        if not self._b:
            raise RuntimeError(te.geterr())

    def run(self):
        return self._L.tcpedit_batch_run(self._te._ctx, self._b)

    def run_fused(self):
        """tcpedit_batch_run with the record discovery fused into the wave lane (window
        mode); batches it does not carry run the exact path, same output"""
        return self._L.tcpedit_batch_run_fused(self._te._ctx, self._b)

    @property
    def fused_fallbacks(self) -> int:
        return int(self._L.tcpedit_batch_fused_fallbacks(self._b))

    def time_fused(self, iters):
        """ms per window-mode run (the wave lane finding its records + the chain check), or
        None when the batch is not one the window mode carries"""
        ms = ctypes.c_double()
        if self._L.tcpedit_batch_time_fused(self._te._ctx, self._b, int(iters), ctypes.byref(ms)) < 0:
            return None
        return ms.value

    def set_prefix(self, recs):
        """the records just before this batch (whole records ending where it starts), read
        by the SURVEY Q8 replay only when a record's stale bytes come from before the batch;
        `recs` is passed by address and must stay alive until the next run returns"""
        keep, p, n = _buf(recs)
        self._prefix_keep = (recs, keep)
        if self._L.tcpedit_batch_set_prefix(self._te._ctx, self._b, p, n) < 0:
            raise RuntimeError(self._te.geterr())

    def update_input(self, pcap):
        """replace the staged image's bytes with `pcap` (same length, same record headers:
        the index and tiles are kept; tcpedit_batch_update_input)"""
        keep, p, n = _buf(pcap)
        if self._L.tcpedit_batch_update_input(self._te._ctx, self._b, p, n) < 0:
            raise RuntimeError(self._te.geterr())

    def result(self) -> BatchResult:
        r = BatchResult()
        self._L.tcpedit_batch_result(self._b, ctypes.byref(r))
        return r

    def output(self) -> bytes:
        r = self.result()
        out = ctypes.create_string_buffer(max(1, r.out_len))
        n = self._L.tcpedit_batch_output(self._b, out, r.out_len)
        return out.raw[:n]

    def output_np(self):
        """the output image as a numpy uint8 array (one D2H copy, no intermediate bytes)"""
        import numpy as np
        r = self.result()
        out = np.empty(max(1, r.out_len), np.uint8)
        n = self._L.tcpedit_batch_output(self._b, out.ctypes.data, r.out_len)
        return out[:n]

    def output_records_into(self, dst) -> int:
        """D2H of the output records (no file header) straight into the writable buffer
        `dst` (a bytearray, or an mmap of the job's output file at this shard's offset);
        returns the bytes written"""
        a, p, n = _buf(dst)
        if n and not a.flags.writeable:
            raise ValueError("dst must be writable")
        return int(self._L.tcpedit_batch_output_records(self._b, p, n))

    def status(self):
        import numpy as np
        r = self.result()
        p = self._L.tcpedit_batch_status(self._b)
        if not p:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array(p, shape=(r.packets,)).copy()

    def fuzz_reach(self) -> int:
        """records of this batch that reach the --fuzz-seed step (tcpedit_batch_fuzz_reach)"""
        n = self._L.tcpedit_batch_fuzz_reach(self._te._ctx, self._b)
        if n < 0:
            raise RuntimeError(self._te.geterr())
        return int(n)

    def l2carry_out(self) -> int:
        """the dst_modified value this batch's last writer leaves (0/1), or 2 when no record
        writes it (tcpedit_batch_l2carry_out)"""
        v = self._L.tcpedit_batch_l2carry_out(self._te._ctx, self._b)
        if v < 0:
            raise RuntimeError(self._te.geterr())
        return int(v)

    def jnpr_out(self):
        """(has one, state bytes): the Juniper decoder state this batch's last whole inner
        decode leaves (tcpedit_batch_jnpr_out), found before any edit"""
        buf = ctypes.create_string_buffer(JNPR_STATE_BYTES)
        v = self._L.tcpedit_batch_jnpr_out(self._te._ctx, self._b, buf, JNPR_STATE_BYTES)
        if v < 0:
            raise RuntimeError(self._te.geterr())
        return v == 1, buf.raw

    def time(self, iters):
        ms = ctypes.c_double()
        if self._L.tcpedit_batch_time(self._te._ctx, self._b, int(iters), ctypes.byref(ms)) < 0:
            raise RuntimeError(self._te.geterr())
        return ms.value

    def time_kernels(self, iters):
        """(ms per run of the whole device pipeline, ms of the edit kernel alone) over `iters` runs"""
        ms, kms = ctypes.c_double(), ctypes.c_double()
        if self._L.tcpedit_batch_time_kernels(self._te._ctx, self._b, int(iters), ctypes.byref(ms),
                                              ctypes.byref(kms)) < 0:
            raise RuntimeError(self._te.geterr())
        return ms.value, kms.value

    def index_device(self, iters=1):
        """rebuild the record index on the device (te_index.hip) -> (applied, device ms per
        build); not applied when the config's tiles are not the wave lane's or a guess
        missed the chain (the host index stays)"""
        ms = ctypes.c_double()
        rc = self._L.tcpedit_batch_index_device(self._te._ctx, self._b, int(iters), ctypes.byref(ms))
        if rc < 0:
            raise RuntimeError(self._te.geterr())
        return rc == 0, ms.value

    def close(self):
        if self._b:
            self._L.tcpedit_batch_close(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
