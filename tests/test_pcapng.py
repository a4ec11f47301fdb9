"""pcapng input: the batch and rewrite calls read a pcapng image
as libpcap's reader hands it to tcprewrite -- classic records at microsecond precision
(te_pcapng.c).  Parity is unpinned (the reference holds no pcapng fixture): the checks
here are that a pcapng file written from a classic capture converts back to it, over the
timestamp resolutions, offsets, byte orders and block kinds libpcap reads, and that the
edit of the pcapng image is the oracle's edit of the classic one."""
import ctypes
import struct

import pytest

import golden_cases as G
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S


def _pad(b):
    return b + bytes(-len(b) % 4)


def _block(e, btype, body):
    n = 12 + len(_pad(body))
    return struct.pack(e + "II", btype, n) + _pad(body) + struct.pack(e + "I", n)


def _opt(e, code, val):
    return struct.pack(e + "HH", code, len(val)) + _pad(val)


def to_pcapng(pcap, e="<", tsresol=None, tsoffset=0, kind="epb", extra_ifs=0, noise=True):
    """a pcapng file with the records of a classic (microsecond) capture: one SHB, an IDB
    (if_tsresol / if_tsoffset), EPB / OPB / SPB records, and blocks libpcap skips"""
    recs = S.records(pcap)
    linktype = struct.unpack_from("<I", pcap, 20)[0]
    units = 10 ** 6
    opts = b""
    if tsresol is not None:
        opts += _opt(e, 9, bytes([tsresol]))
        units = 2 ** (tsresol & 0x7F) if tsresol & 0x80 else 10 ** tsresol
    if tsoffset:
        opts += _opt(e, 14, struct.pack(e + "q", tsoffset))
    if opts:
        opts += _opt(e, 0, b"")
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += _block(e, 1, struct.pack(e + "HHI", linktype, 0, 262144) + opts)
    for _ in range(extra_ifs):
        out += _block(e, 1, struct.pack(e + "HHI", linktype, 0, 65535))
    if noise:
        out += _block(e, 4, b"\x00\x00\x00\x00")  # a name resolution block: skipped
    for ts, tu, cl, ln, d in recs:
        t = (ts - tsoffset) * units + -(-tu * units // 10 ** 6)  # (ceiling: the reader truncates)
        if kind == "epb":
            out += _block(e, 6, struct.pack(e + "IIIII", 0, t >> 32, t & 0xFFFFFFFF, cl, ln) + d)
        elif kind == "opb":
            out += _block(e, 2, struct.pack(e + "HHIIII", 0, 0, t >> 32, t & 0xFFFFFFFF, cl, ln) + d)
    if noise:
        out += _block(e, 5, struct.pack(e + "III", 0, 0, 0))  # interface statistics: skipped
    return out


def _convert(img):
    L = ctypes.CDLL(TA.LIB_PATH)
    L.tcpedit_pcapng_to_pcap.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_size_t)]
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = L.tcpedit_pcapng_to_pcap(img, len(img), ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        return None
    data = ctypes.string_at(out, n.value)
    ctypes.CDLL("libc.so.6").free(out)
    return data


def _classic(pcap):
    """the classic capture as the conversion writes its header: LE, microseconds, v2.4,
    the IDB's snaplen (262144 here) and link type"""
    return struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 262144, 1) + pcap[24:]


@pytest.mark.parametrize("e,tsresol,tsoffset,kind", [
    ("<", None, 0, "epb"), (">", None, 0, "epb"), ("<", 9, 0, "epb"), ("<", 3, 0, "epb"),
    (">", 0x80 | 20, 0, "epb"), ("<", 6, 1_000_000_000, "epb"), ("<", None, 0, "opb"), (">", 9, 7, "opb"),
])
def test_pcapng_converts_to_the_classic_records(built, e, tsresol, tsoffset, kind):
    pcap = G.read("test.pcap")
    if tsresol == 3:  # millisecond clock: the microseconds below a millisecond are gone
        recs = [(ts, tu - tu % 1000, cl, ln, d) for ts, tu, cl, ln, d in S.records(pcap)]
        pcap = S.build_pcap(recs)
    assert _convert(to_pcapng(pcap, e, tsresol, tsoffset, kind)) == _classic(pcap)


def test_simple_packet_blocks_take_the_snaplen(built):
    recs = S.records(S.pcap_fixed(20, 200, seed=3))
    e = "<"
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += _block(e, 1, struct.pack(e + "HHI", 1, 0, 100))
    for ts, tu, cl, ln, d in recs:
        out += _block(e, 3, struct.pack(e + "I", ln) + d)
    got = S.records(_convert(out))
    assert [(r[0], r[1], r[2], r[3]) for r in got] == [(0, 0, 100, 200)] * 20
    assert [r[4] for r in got] == [d[:100] for *_, d in recs]


def test_mixed_link_types_and_garbage_are_refused(built):
    pcap = G.read("test.pcap")
    ng = to_pcapng(pcap)
    e = "<"
    bad = ng + _block(e, 1, struct.pack(e + "HHI", 101, 0, 65535))  # a raw-IP interface after Ethernet
    assert _convert(bad) is None
    assert _convert(b"\x0a\x0d\x0d\x0a" + bytes(40)) is None


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["--seed=42", "--fixcsum"], ["--enet-vlan=add", "--enet-vlan-tag=9"],
                                  ["--pnat=10.0.0.0/8:192.168.0.0/16", "--efcs"]])
def test_gpu_rewrites_pcapng_as_the_classic_capture(built, args):
    pcap = S.pcap_imix(20_000, seed=5)
    ng = to_pcapng(pcap, ">", 9, 0, "epb")
    _, exp = O.rewrite(_classic(pcap), args)
    te = TA.TcpEdit(args)
    try:
        rc, out = te.rewrite(ng)
        assert rc == 0 and out == exp
        rc, out = te.rewrite_pipelined(ng, chunk_bytes=1 << 20)
        assert rc == 0 and out == exp
    finally:
        te.close()


@pytest.mark.parametrize("ifn", [1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF])
def test_epb_interface_id_out_of_range_is_refused(built, ifn):
    """an EPB naming an interface the section never described is a malformed block (the id
    is compared unsigned: 0x80000000 and up must not pass as negative)"""
    e = "<"
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += _block(e, 1, struct.pack(e + "HHI", 1, 0, 65535))
    out += _block(e, 6, struct.pack(e + "IIIII", ifn, 0, 0, 60, 60) + bytes(60))
    assert _convert(out) is None


def test_epb_captured_length_past_the_block_is_refused(built):
    e = "<"
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += _block(e, 1, struct.pack(e + "HHI", 1, 0, 65535))
    out += _block(e, 6, struct.pack(e + "IIIII", 0, 0, 0, 0xFFFFFFF0, 60) + bytes(60))
    assert _convert(out) is None


@pytest.mark.parametrize("snaplen,want", [(100, 100), (0, 1514), (1 << 20, 1514)])
def test_records_are_cut_to_the_snapshot_length(built, snaplen, want):
    """libpcap's pcap-ng reader cuts a record whose captured length exceeds the capture's
    snapshot length (the first IDB's snaplen; 0 or more than 262144 meaning 262144) to it.
    Stated from libpcap's behaviour; parity unpinned (no reference pcapng fixture)."""
    recs = S.records(S.pcap_fixed(5, 1514, seed=4))
    e = "<"
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    out += _block(e, 1, struct.pack(e + "HHI", 1, 0, snaplen))
    for ts, tu, cl, ln, d in recs:
        out += _block(e, 6, struct.pack(e + "IIIII", 0, 0, 0, cl, ln) + d)
    got = S.records(_convert(out))
    assert [(r[2], r[3]) for r in got] == [(want, 1514)] * 5
    assert [r[4] for r in got] == [d[:want] for *_, d in recs]
