"""Python mirror of tcpreplay's replay passes with --unique-ip (include/tcpreplay_hip.h).

Same option names as the reference's tcpreplay (src/tcpreplay_opts.def, long forms) for
the options this path serves -- --loop, --unique-ip, --unique-ip-loops, --preload-pcap
(-K) -- and the same output as `tcpreplay -w <file>`: every pass over the capture, each
record as sendpacket's pcap dump writes it.  fast_edit_packet (send_packets.c:124-257)
runs in the tr_mark kernel of libtcpedit_hip.so; there is no CPU path.
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
                ("tcpreplay_hip_init", vp, []),
                ("tcpreplay_hip_close", None, [vp]),
                ("tcpreplay_hip_geterr", ctypes.c_char_p, [vp]),
                ("tcpreplay_hip_parse_args", c_int, [vp, c_int, ctypes.POINTER(ctypes.c_char_p)]),
                ("tcpreplay_hip_set_loop", c_int, [vp, ctypes.c_uint32]),
                ("tcpreplay_hip_set_unique_ip", c_int, [vp, ctypes.c_bool]),
                ("tcpreplay_hip_set_unique_ip_loops", c_int, [vp, c_int]),
                ("tcpreplay_hip_set_preload_pcap", c_int, [vp, ctypes.c_bool]),
                ("tcpreplay_hip_output_bound", sz, [vp, sz]),
                ("tcpreplay_hip_replay_to_pcap", ctypes.c_int64,
                 [vp, ctypes.c_char_p, sz, vp, sz, ctypes.POINTER(ctypes.c_uint64)]),
                ("tcpreplay_hip_reader_exited", c_int, [vp]),
                ("tcpreplay_hip_output_len", ctypes.c_int64, [vp])):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _SIG_DONE = True
    return L


READER_EXIT = -2  # TCPREPLAY_HIP_READER_EXIT


class ReaderExit(RuntimeError):
    """the replay ended where safe_pcap_next exit(-1)s (src/common/utils.c:136-156): `output`
    is the -w file tcpreplay wrote before exiting, `failed` its failed unique-ip edits"""

    def __init__(self, msg, output, failed):
        super().__init__(msg)
        self.output, self.failed = output, failed


class TcpReplay:
    """tcpreplay_hip_init + tcpreplay_hip_parse_args; replay(pcap) -> (the -w file bytes,
    the records whose unique-ip edit failed: stats->failed); a run that ends at
    safe_pcap_next's exit raises ReaderExit (its partial output attached)"""

    def __init__(self, args):
        self._L = _lib()
        self._ctx = self._L.tcpreplay_hip_init()
        if not self._ctx:
            raise MemoryError("tcpreplay_hip_init failed")
        argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
        if self._L.tcpreplay_hip_parse_args(self._ctx, len(args), argv) != 0:
            err = self.geterr()
            self.close()
            raise ValueError(err)

    def geterr(self):
        e = self._L.tcpreplay_hip_geterr(self._ctx)
        return e.decode() if e else ""

    def replay(self, pcap: bytes):
        cap = self._L.tcpreplay_hip_output_bound(self._ctx, len(pcap))
        out = ctypes.create_string_buffer(max(cap, 1))
        failed = ctypes.c_uint64()
        n = self._L.tcpreplay_hip_replay_to_pcap(self._ctx, pcap, len(pcap), out, cap, ctypes.byref(failed))
        if n == READER_EXIT:
            raise ReaderExit(self.geterr(), out.raw[:self._L.tcpreplay_hip_output_len(self._ctx)], int(failed.value))
        if n < 0:
            raise RuntimeError(self.geterr())
        return out.raw[:n], int(failed.value)

    @property
    def reader_exited(self) -> bool:
        """the last replay ended at safe_pcap_next's exit (src/common/utils.c:136-156): its
        output is what tcpreplay wrote before exiting"""
        return bool(self._L.tcpreplay_hip_reader_exited(self._ctx))

    def close(self):
        if self._ctx:
            self._L.tcpreplay_hip_close(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def replay(pcap: bytes, args):
    t = TcpReplay(args)
    try:
        return t.replay(pcap)
    finally:
        t.close()
