"""ctypes loader for the CPU oracle (oracle/_build/liboracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        lib = ctypes.CDLL(LIB_PATH)
        lib.oracle_rewrite_mem.restype = ctypes.c_int
        lib.oracle_rewrite_mem.argtypes = [
            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
            ctypes.POINTER(ctypes.c_char_p), ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
        lib.oracle_mix_seed.restype = ctypes.c_uint32
        lib.oracle_mix_seed.argtypes = [ctypes.c_uint32]
        lib.oracle_warn_count.restype = ctypes.c_int
        lib.oracle_fuzz_draws.restype = ctypes.c_uint64
        lib.oracle_set_fuzz_skip.argtypes = [ctypes.c_uint64]
        lib.oracle_set_fuzz_skip.restype = None
        _lib = lib
    return _lib


def rewrite(pcap: bytes, args, cache: bytes = None, want_status=False):
    """Run the oracle over an in-memory pcap.  Returns (rc, output_bytes[, status])."""
    lib = load()
    argv = (ctypes.c_char_p * max(1, len(args)))(*[a.encode() for a in args])
    # worst-case growth: +4 B per record (VLAN add) or fixlen pad up to len
    cap = len(pcap) * 2 + 1024 + 262144
    out = ctypes.create_string_buffer(cap)
    out_len = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(1024)
    inbuf = ctypes.create_string_buffer(pcap, len(pcap))
    cbuf = ctypes.create_string_buffer(cache, len(cache)) if cache else None
    npk = max(1, len(pcap) // 16)
    status = np.zeros(npk, dtype=np.int8)
    rc = lib.oracle_rewrite_mem(inbuf, len(pcap), cbuf, len(cache) if cache else 0, len(args), argv, out, cap,
                                ctypes.byref(out_len), status.ctypes.data, npk, err, 1024)
    data = out.raw[:out_len.value]
    if rc == -2:
        raise ValueError("oracle rejected input/options: " + err.value.decode(errors="replace"))
    if want_status:
        return rc, data, status
    return rc, data


def mix_seed(seed: int) -> int:
    return load().oracle_mix_seed(seed)


def fuzz_draws() -> int:
    """tcpr_random() draws the last rewrite() made for --fuzz-seed"""
    return int(load().oracle_fuzz_draws())


def rewrite_skipping(pcap: bytes, args, cache: bytes = None, skip: int = 0):
    """rewrite() with the --fuzz-seed stream advanced by `skip` draws first (a shard)"""
    lib = load()
    lib.oracle_set_fuzz_skip(int(skip))
    try:
        return rewrite(pcap, args, cache)
    finally:
        lib.oracle_set_fuzz_skip(0)


def tcpprep(pcap: bytes, args, pkt_base: int = 0, with_entries=False):
    """tcpprep_oracle_run: the CPU restatement of tcpprep's per-packet modes -> cache file
    bytes (and the entry count).  pkt_base = a shard's first global record number."""
    lib = load()
    lib.tcpprep_oracle_set_pkt_base.argtypes = [ctypes.c_uint64]
    lib.tcpprep_oracle_set_pkt_base.restype = None
    lib.tcpprep_oracle_last_entries.restype = ctypes.c_uint64
    lib.tcpprep_oracle_set_pkt_base(int(pkt_base))
    fn = lib.tcpprep_oracle_run
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.c_char_p, ctypes.c_size_t,
                   ctypes.c_char_p, ctypes.c_size_t]
    argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
    cap = 24 + 8192 + len(pcap) // 16 + 64
    out = ctypes.create_string_buffer(cap)
    n = fn(len(args), argv, pcap, len(pcap), out, cap)
    lib.tcpprep_oracle_set_pkt_base(0)
    if n < 0:
        raise ValueError(f"tcpprep oracle failed ({n}) for {args}")
    if with_entries:
        return out.raw[:n], int(lib.tcpprep_oracle_last_entries())
    return out.raw[:n]


def replay_args(args, with_list=False):
    """tcpreplay's options this path serves (tcpreplay_opts.def): --loop, --unique-ip,
    --unique-ip-loops, --preload-pcap / -K, --include / --exclude -> (loops, unique_ip,
    unique_loops, preload[, list, exclude])"""
    loops, uniq, uloops, preload, lst, excl = 1, 0, 1.0, 0, None, 0
    for a in args:
        k, _, v = a.partition("=")
        if k in ("--loop", "-l"):
            loops = int(v)
        elif k == "--unique-ip":
            uniq = 1
        elif k == "--unique-ip-loops":
            uloops = float(v)
        elif k in ("--preload-pcap", "-K"):
            preload = 1
        elif k in ("--include", "--exclude"):
            if lst is not None:
                raise ValueError("--include and --exclude: one list")
            lst, excl = v, int(k == "--exclude")
        else:
            raise ValueError(f"unknown tcpreplay option {a}")
    return (loops, uniq, uloops, preload, lst, excl) if with_list else (loops, uniq, uloops, preload)


def replay(pcap: bytes, args):
    """tcpreplay_oracle_run: `tcpreplay -w out <args> <pcap>` as the CPU restatement writes
    it -> (output file bytes, records whose unique-ip edit failed)"""
    lib = load()
    fn = lib.tcpreplay_oracle_run_list
    fn.restype = ctypes.c_long
    fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                   ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]
    loops, uniq, uloops, preload, lst, excl = replay_args(args, with_list=True)
    cap = 24 + loops * max(len(pcap) - 24, 0) + 64
    out = ctypes.create_string_buffer(cap)
    failed = ctypes.c_uint64()
    n = fn(pcap, len(pcap), loops, uniq, uloops, preload, lst.encode() if lst is not None else None, excl, out, cap,
           ctypes.byref(failed))
    if n < 0:
        raise ValueError(f"tcpreplay oracle failed ({n}) for {args}")
    return out.raw[:n], int(failed.value)


def replay_edit(pcap: bytes, args, loops=1, preload=False):
    """tcpreplay_edit_oracle_run: `tcpreplay-edit -w out --loop=loops [-K] <args> in.pcap`
    restated on the CPU.  Returns (rc, the -w file's bytes); rc -1 = the run's errx (the
    records sent before it kept), ValueError for what the restatement refuses."""
    lib = load()
    fn = lib.tcpreplay_edit_oracle_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_char_p), ctypes.c_void_p, ctypes.c_size_t,
                   ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_int]
    argv = (ctypes.c_char_p * max(1, len(args)))(*[a.encode() for a in args])
    cap = 24 + max(1, loops) * (2 * len(pcap) + 1024 + 262144)
    out = ctypes.create_string_buffer(cap)
    out_len = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(1024)
    inbuf = ctypes.create_string_buffer(pcap, len(pcap))
    rc = fn(inbuf, len(pcap), int(loops), 1 if preload else 0, len(args), argv, out, cap, ctypes.byref(out_len),
            err, 1024)
    if rc == -2:
        raise ValueError("oracle rejected input/options: " + err.value.decode(errors="replace"))
    return rc, out.raw[:out_len.value]


def replay_edit_failed() -> int:
    """records whose --unique-ip edit failed in the last replay_edit (stats->failed)"""
    fn = load().tcpreplay_edit_oracle_failed
    fn.restype = ctypes.c_uint64
    return int(fn())


def check_rewrite(pcap, args, cache, dev_out, threads=16, sharded=True, pkt_base=0):
    """The checker bench.py runs outside its timed region: the oracle's tcprewrite output
    for (pcap, args, cache) must equal `dev_out` (the device's output image, any
    bytes-like object) byte for byte.  With `sharded` the records are cut into `threads`
    byte-balanced runs, each rewritten by the oracle on its own thread at its global record
    number (oracle_rewrite_mem_base); only valid when records are independent (no
    --fuzz-seed, no stale static-buffer reads).  `pkt_base`: the capture's first record is
    record pkt_base of the job (a shard), for the tcpprep cache lookups.  Returns the records checked; raises
    AssertionError naming the first differing run."""
    from concurrent.futures import ThreadPoolExecutor
    lib = load()
    fn = lib.oracle_rewrite_mem_base
    fn.restype = ctypes.c_int
    fn.argtypes = lib.oracle_rewrite_mem.argtypes + [ctypes.c_uint64]
    cutf = lib.oracle_shard_cuts
    cutf.restype = ctypes.c_uint64
    cutf.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    src = np.frombuffer(pcap, np.uint8)
    dev = np.frombuffer(dev_out, np.uint8)
    parts = max(1, int(threads)) if sharded else 1
    cuts = np.zeros(parts + 1, np.uint64)
    first = np.zeros(parts + 1, np.uint64)
    nrec = int(cutf(src.ctypes.data, src.size, parts, cuts.ctypes.data, first.ctypes.data))
    argv = (ctypes.c_char_p * max(1, len(args)))(*[a.encode() for a in args])
    cbuf = np.frombuffer(cache, np.uint8) if cache else None
    hdr = src[:24]

    def one(k):
        a, b = int(cuts[k]), int(cuts[k + 1])
        if b <= a and k > 0:
            return k, 0, None, None
        if parts == 1:  # the whole capture, trailing bytes and all
            shard = src
        else:
            shard = np.empty(24 + b - a, np.uint8)
            shard[:24] = hdr
            shard[24:] = src[a:b]
        cap = 2 * shard.size + 1024 + 262144
        out = np.empty(cap, np.uint8)
        olen = ctypes.c_size_t(0)
        err = ctypes.create_string_buffer(1024)
        rc = fn(shard.ctypes.data, shard.size, cbuf.ctypes.data if cbuf is not None else None,
                cbuf.size if cbuf is not None else 0, len(args), argv, out.ctypes.data, cap, ctypes.byref(olen),
                None, 0, err, 1024, int(pkt_base) + int(first[k]))
        return k, rc, out[:olen.value], err.value.decode(errors="replace")

    pos = 24
    with ThreadPoolExecutor(max_workers=parts) as ex:
        for k, rc, out, err in ex.map(one, range(parts)):
            if out is None:
                continue
            if rc != 0:
                raise AssertionError(f"oracle run {k} failed rc={rc}: {err}")
            if k == 0 and bytes(dev[:24]) != bytes(out[:24]):
                raise AssertionError("output file header differs from the oracle's")
            body = out[24:]
            seg = dev[pos:pos + body.size]
            if seg.size != body.size or not np.array_equal(seg, body):
                bad = np.flatnonzero(seg != body[:seg.size])
                where = int(bad[0]) if bad.size else min(seg.size, body.size)
                raise AssertionError(f"device output differs from the oracle in run {k} (records from "
                                     f"{int(first[k])}): output byte {pos + where}")
            pos += body.size
    if pos != dev.size:
        raise AssertionError(f"device output is {dev.size} bytes, the oracle's {pos}")
    return nrec
