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
                ("tcpprep_close", c_int, [ctypes.POINTER(vp)])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _SIG_DONE = True
    return L


class TcpPrep:
    """tcpprep_init + tcpprep_parse_args; cache(pcap) -> cache file bytes."""

    def __init__(self, args):
        self._L = _lib()
        self._ctx = ctypes.c_void_p()
        if self._L.tcpprep_init(ctypes.byref(self._ctx)) != 0:
            raise MemoryError("tcpprep_init failed")
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
