"""The generic lane's per-record edit on the host (CPU suite, no GPU).

tests/emu/te_emu.cpp compiles the device edit (edit_pkt.hpp tcpedit_packet, the code
te_edit_tiles runs one lane per record) for the host with AddressSanitizer and UBSan and
lays each record out in its own heap slot exactly as the kernel's tile body does: the
config's headroom (te_dev_cfg_t.slot_head), the alignment gap, the record, 16 zeroed
bytes.  Driving it over the option lines here checks the device logic against the
oracle record by record before a GPU runs it, and turns a move of the record header
past its slot into a sanitizer report instead of an LDS overwrite (the
fuzz + any-decoder instance faulted on the box because the second encode of a fuzzed
record -- tcpedit.c:89,250-258 -- moved the header past the headroom one call at a time
checked).  Test infrastructure only: the product never loads the emulator.

Parity of the non-Ethernet framings is unpinned (the reference ships no capture of
them): the oracle restates the reference's plugins, and the GPU tests check the device
against the oracle on the same lines."""
import ctypes
import os
import subprocess

import pytest

import oracle_lib as O
import tcpreplay_amd as TA
from cfg_struct import DevCfg
from tcpreplay_amd import synth as S

HERE = os.path.dirname(os.path.abspath(__file__))
EMU = os.path.join(HERE, "emu", "_build", "te_emu")
DLT_OF = {"sll": 113, "sll2": 276, "raw": 12, "raw12": 12, "null": 0, "loop": 108, "ppp": 50, "chdlc": 104}
DEC_L2 = {1: 14, 113: 16, 276: 20, 12: 0, 0: 4, 108: 4, 50: 4, 104: 4, 178: 6, 105: 24, 127: 24}
MACS = ["--enet-smac=00:11:22:33:44:55,00:aa:bb:cc:dd:ee", "--enet-dmac=00:66:77:88:99:aa,00:12:34:56:78:9a"]
USER14 = ["--dlt=user", "--user-dlink=01,02,03,04,05,06,07,08,09,0a,0b,0c,08,00", "--user-dlt=1"]
USER40 = ["--dlt=user", "--user-dlink=" + ",".join("%02x" % (b + 0x40) for b in range(38)) + ",08,00",
          "--user-dlt=1"]

FUZZ_LINES = [
    ["--dlt=enet"] + MACS + ["--fuzz-seed=7", "--fuzz-factor=2", "--fixcsum"],
    USER14 + ["--fuzz-seed=5", "--fuzz-factor=3"],
    USER40 + ["--fuzz-seed=11", "--fuzz-factor=1", "--fixcsum"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--fuzz-seed=9", "--fuzz-factor=2"],
    ["--fuzz-seed=3", "--fuzz-factor=1"],  # the decoder's own plugin as the encoder
]
PLAIN_LINES = [
    ["--fixcsum"],
    ["--dlt=enet"] + MACS + ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353", "--fixcsum"],
    ["--dlt=enet"] + MACS + ["--enet-vlan=del", "--tos=5", "--mtu-trunc", "--mtu=400", "--fixcsum"],
    USER14 + ["--fixcsum"],
    USER40 + ["--seed=4", "--fixcsum"],
    ["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=3", "--seed=5"],
]
ETH_LINES = [
    ["--seed=42", "--fixcsum"],
    ["--fuzz-seed=42", "--fuzz-factor=2"],
    ["--fuzz-seed=42", "--fuzz-factor=1", "--enet-vlan=add", "--enet-vlan-tag=9", "--fixcsum"],
    ["--fuzz-seed=8", "--fuzz-factor=1", "--mtu-trunc", "--mtu=300", "--fixlen=pad"],
    USER40 + ["--fuzz-seed=6", "--fuzz-factor=1"],
    ["--dlt=hdlc", "--hdlc-address=1", "--hdlc-control=2", "--fuzz-seed=2", "--fuzz-factor=1", "--fixcsum"],
]


@pytest.fixture(scope="module")
def emu(built):
    # one build at a time (pytest -n: every worker asks for it), under a lock file
    import fcntl
    os.makedirs(os.path.dirname(EMU), exist_ok=True)
    with open(EMU + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "emu")])
    return EMU


def _cfg(args, dlt):
    te = TA.TcpEdit(args, dlt=dlt)
    try:
        cfg = DevCfg()
        lut = (ctypes.c_uint16 * 65536)()
        n = te._L.tcpedit_get_dev_cfg(te._ctx, ctypes.byref(cfg), ctypes.sizeof(cfg), lut)
        assert n == ctypes.sizeof(cfg)
        return cfg, bytes(lut)
    finally:
        te.close()


def _grows(cfg, dlt):
    dl = DEC_L2.get(dlt, 14)
    if cfg.encoder == 1:
        return cfg.user_length - dl > 0
    if cfg.encoder == 2:
        return 4 - dl > 0
    return (cfg.encoder == 0 and cfg.vlan == 2) or (cfg.encoder == 0 and dlt != 1 and 14 - dl > 0) or cfg.fixlen == 1


def _emu_run(emu, tmp, pcap, args, dlt, slot, cache=None):
    cfg, lut = _cfg(args, dlt)
    paths = {k: os.path.join(tmp, k) for k in ("cfg", "lut", "in", "dir", "out")}
    for k, v in (("cfg", bytes(cfg)), ("lut", lut), ("in", pcap), ("dir", cache)):
        if v is not None:
            with open(paths[k], "wb") as f:
                f.write(v)
    dirarg = "-"
    if cache is not None:
        hl = 24 + int.from_bytes(cache[20:22], "big")  # tcpprep v04 header + comment
        with open(paths["dir"], "wb") as f:
            f.write(cache[hl:])
        dirarg = paths["dir"]
    r = subprocess.run([emu, paths["cfg"], paths["lut"], paths["in"], dirarg, str(slot), paths["out"]],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    stats = dict(zip(r.stdout.split()[0::2], (int(x) for x in r.stdout.split()[1::2])))
    with open(paths["out"], "rb") as f:
        return stats, f.read(), cfg


def _check(emu, tmp, pcap, args, dlt, cache=None):
    rc_o, exp = O.rewrite(pcap, args, cache)
    cfg, _ = _cfg(args, dlt)
    for slot in ([1] if _grows(cfg, dlt) else [0, 1]):
        stats, out, _ = _emu_run(emu, tmp, pcap, args, dlt, slot, cache)
        # no record needs the Q8 replay (these captures have no stale-buffer reads), and
        # none ran out of headroom (that would flag it the same way)
        assert stats["unsupported"] == 0, (args, slot, stats)
        assert (stats["error"] != 0) == (rc_o != 0), (args, slot, stats, rc_o)
        assert S.records(out) == S.records(exp), (args, slot)


@pytest.mark.parametrize("kind", list(DLT_OF))
@pytest.mark.parametrize("k", range(len(FUZZ_LINES)))
def test_emu_fuzz_behind_every_decoder(emu, tmp_path, kind, k):
    """--fuzz-seed behind every decoder into every encoder: the device edit, laid out in
    its slot, equals the oracle, and no record leaves its slot"""
    pcap = S.reframe(S.pcap_imix(1200, seed=k + 21), kind, odd_every=9)
    _check(emu, str(tmp_path), pcap, FUZZ_LINES[k], DLT_OF[kind])


@pytest.mark.parametrize("kind", list(DLT_OF))
@pytest.mark.parametrize("k", range(len(PLAIN_LINES)))
def test_emu_decoders(emu, tmp_path, kind, k):
    pcap = S.reframe(S.pcap_imix(800, seed=k + 3), kind, odd_every=11)
    _check(emu, str(tmp_path), pcap, PLAIN_LINES[k], DLT_OF[kind])


@pytest.mark.parametrize("kind", ["jnpr", "80211", "radiotap"])
@pytest.mark.parametrize("k", range(len(FUZZ_LINES)))
def test_emu_fuzz_behind_wireless_decoders(emu, tmp_path, kind, k):
    pcap = S.reframe(S.pcap_imix(1200, seed=k + 31), kind, odd_every=9)
    _check(emu, str(tmp_path), pcap, FUZZ_LINES[k], S.LINKTYPES_MORE[kind])


@pytest.mark.parametrize("k", range(len(ETH_LINES)))
def test_emu_ethernet(emu, tmp_path, k):
    """Ethernet input: fuzzing with a VLAN push (two pushes for a fuzzed record, Q11), with
    --fixlen=pad and --mtu-trunc, and into a 40-byte user header (headroom 2 x 26)"""
    pcap = S.pcap_imix(1500, seed=k + 5)
    _check(emu, str(tmp_path), pcap, ETH_LINES[k], 1)


@pytest.mark.parametrize("k", range(5))
def test_emu_jnpr_warning_frames(emu, tmp_path, k):
    """Juniper frames whose extensions are not Ethernet (TCPEDIT_WARN), encoded with the
    carried decoder state -- plain and fuzzed lines, into en10mb, user and hdlc"""
    import test_dlt_wireless as W
    lines = [W.JNPR_LINES[0], W.JNPR_LINES[1], W.JNPR_LINES[3], W.JNPR_LINES[4], W.JNPR_LINES[5]]
    pcap, _ = W._jnpr_warn(1500, seed=k + 41)
    _check(emu, str(tmp_path), pcap, lines[k], 178)


@pytest.mark.parametrize("k", range(2))
def test_emu_jnpr_second_decode_is_a_warning_frame(emu, tmp_path, k):
    """a fuzzed record's second decode taken by the Juniper decoder as a warning frame (the
    re-encoded frame starts with the Juniper magic: --enet-dmac 4d:47:43:80:00:00) reads the
    state its own first pass left (tests/test_dlt_wireless.py, GPU)"""
    import test_dlt_wireless as W
    pcap, _ = W._jnpr_warn(1200, seed=k + 61)
    args = ["--dlt=enet", "--enet-dmac=" + W.JMAGIC_DMAC, "--enet-smac=00:11:22:33:44:55",
            "--fuzz-seed=%d" % (k + 5), "--fuzz-factor=%d" % (k + 2)]
    _check(emu, str(tmp_path), pcap, args, 178)


def test_emu_headroom_holds_two_encodes(emu, tmp_path):
    """the config's headroom covers both encodes of a fuzzed record (te_slot_head)"""
    cfg, _ = _cfg(USER40 + ["--fuzz-seed=1"], 12)
    assert cfg.slot_head >= 2 * 40 and cfg.slot_head % 16 == 0
    cfg, _ = _cfg(["--fixcsum"], 1)
    assert cfg.slot_head == 16
