"""CPU tests of the native library's host side: it loads, exports the whole
C-ABI declared in include/tcpedit.h, and derives the per-run device tables
(tcpedit_post_args, parse_args.c:34-254; en10mb.c:226-396) exactly.
No kernel is launched here."""
import ctypes
import os
import re
import socket
import struct

import numpy as np
import pytest

import tcpreplay_amd as TA
from cfg_struct import DevCfg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(header="tcpedit.h", prefix="tcpedit_"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(built):
    L = ctypes.CDLL(TA.LIB_PATH)
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert missing == []


def test_library_exports_every_tcpprep_symbol(built):
    L = ctypes.CDLL(TA.LIB_PATH)
    names = header_functions("tcpprep.h", "tcpprep_")
    assert len(names) == 12
    assert [n for n in names if not hasattr(L, n)] == []


def test_library_exports_every_tcpreplay_symbol(built):
    L = ctypes.CDLL(TA.LIB_PATH)
    names = header_functions("tcpreplay_hip.h", "tcpreplay_hip_")
    assert len(names) == 12
    assert [n for n in names if not hasattr(L, n)] == []


def derive(args):
    te = TA.TcpEdit(args)
    cfg = DevCfg()
    lut = (ctypes.c_uint16 * 65536)()
    n = te._L.tcpedit_get_dev_cfg(te._ctx, ctypes.byref(cfg), ctypes.sizeof(cfg), lut)
    assert n == ctypes.sizeof(cfg)
    return te, cfg, np.frombuffer(lut, np.uint16).copy()


def tcpr_random(seed):
    n = seed & 0xFFFFFFFF

    def step(n):
        return (n * 1103515245 + 12345) & 0xFFFFFFFF
    n = step(n)
    r = (n // 65536) % 2048
    n = step(n)
    r = ((r << 10) ^ ((n // 65536) % 1024)) & 0xFFFFFFFF
    n = step(n)
    r = ((r << 10) ^ ((n // 65536) % 1024)) & 0xFFFFFFFF
    return n, r


def mix(seed, k=5):
    r = 0
    for _ in range(k):
        seed, r = tcpr_random(seed)
    return seed, r


def nport(p):
    return struct.unpack("<H", struct.pack(">H", p))[0]  # port as loaded LE from packet bytes


def test_seed_and_sequence(built):
    _, c, _ = derive(["--seed=42", "--tcp-sequence=42"])
    assert c.seed == 0x75B59D85 == mix(42)[0]
    assert c.rewrite_ip == 1
    assert c.tcp_sequence_enable == 1 and c.tcp_sequence_adjust == mix(42)[1]


def test_portmap_first_match_lut(built):
    _, c, lut = derive(["--portmap=80:8080,81+82:9000", "-r", "1-3:49148", "--portmap=80:1"])
    assert c.has_portmap == 1
    assert lut[nport(80)] == nport(8080)          # first record wins over the later 80:1
    assert lut[nport(81)] == nport(9000) and lut[nport(82)] == nport(9000)
    assert [lut[nport(p)] for p in (1, 2, 3)] == [nport(49148)] * 3
    assert lut[0] == 0 and lut[nport(4)] == nport(4)


def test_portmap_bad_first_record_is_error(built):
    with pytest.raises(ValueError):
        derive(["--portmap=x:1"])


def test_portmap_bad_later_record_is_dropped(built):
    _, c, lut = derive(["--portmap=80:8080,zz:1,90:91"])  # portmap.c:198-214
    assert lut[nport(80)] == nport(8080) and lut[nport(90)] == nport(91)


def ipn(s):
    return struct.unpack("<I", socket.inet_aton(s))[0]


def test_pnat_and_endpoints(built):
    _, c, _ = derive(["--pnat=96.17.211.0/24:172.16.0.0/24"])
    assert c.n_cidrmap1 == 1 and c.n_cidrmap2 == 1  # one -N serves both directions
    m = c.cidrmap1[0]
    assert (m.frm.family, m.frm.masklen, m.frm.network) == (4, 24, ipn("96.17.211.0"))
    assert (m.to.family, m.to.masklen, m.to.network) == (4, 24, ipn("172.16.0.0"))
    _, c, _ = derive(["--endpoints=10.10.0.1:10.10.0.2"])
    assert c.cidrmap1[0].frm.masklen == 0 and c.cidrmap1[0].to.network == ipn("10.10.0.1")
    assert c.cidrmap2[0].to.network == ipn("10.10.0.2") and c.cidrmap2[0].to.masklen == 32
    _, c, _ = derive(["--pnat=[::/0]:[2001:db8:aaaa::/36]"])
    assert c.cidrmap1[0].to.family == 6 and c.cidrmap1[0].to.masklen == 36
    assert bytes(c.cidrmap1[0].to.network6) == socket.inet_pton(socket.AF_INET6, "2001:db8:aaaa::")


def test_l2_options(built):
    _, c, _ = derive(["--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-cfi=1", "--enet-vlan-pri=5",
                      "--enet-vlan-proto=802.1ad",
                      "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66", "--enet-smac=,00:12:13:14:15:16"])
    assert (c.vlan, c.vlan_tag, c.vlan_cfi, c.vlan_pri, c.vlan_proto) == (2, 45, 1, 5, 0x88A8)
    # strtok_r skips the empty leading field, so ",X" sets the FIRST mac (mac.c:84-98)
    assert c.mac_mask == 4 | 8 | 1
    assert bytes(c.intf2_dmac) == bytes.fromhex("002233445566")
    _, c, _ = derive(["--enet-subsmac=00:1f:f3:3c:e1:13,00:22:33:44:55:66",
                      "--enet-subsmac=f8:1e:df:e5:84:3a,00:66:55:44:33:22,01:02:03:04:05:06,0a:0b:0c:0d:0e:0f"])
    assert c.n_subs == 3
    assert bytes(c.subs[2]) == bytes.fromhex("0102030405060a0b0c0d0e0f")
    _, c, _ = derive(["--enet-mac-seed=42", "--enet-mac-seed-keep-bytes=3"])
    st, masks = 42, []
    while len(masks) < 6:
        st, r = tcpr_random(st)
        if (r & 0xFF) not in masks:
            masks.append(r & 0xFF)
    assert list(c.random_mask[:6]) == masks and c.random_keep == 3 and c.random_set == st


@pytest.mark.parametrize("args", [
    ["--fixlen=foo"], ["--ttl=300"], ["--enet-vlan=add"], ["--enet-vlan=bogus"], ["--tos=256"],
    ["--seed=1", "--fuzz-seed=2"], ["--pnat=1.2.3.0/24:5.6.7.0/24", "--srcipmap=1.0.0.0/8:2.0.0.0/8"],
    ["--enet-mac-seed=1", "--enet-smac=00:00:00:00:00:01"], ["--enet-vlan-tag=4"], ["--mtu=0"],
    ["--pnat=1.2.3.4"], ["--pnat=300.1.1.1/8:1.1.1.1/8"], ["--dlt=user"], ["--nonsense"], ["--seed=1", "-s", "2"],
])
def test_invalid_options_are_rejected(built, args):
    with pytest.raises(ValueError):
        derive(args)


def test_ttl_modes(built):
    for a, mode, val in (("58", 1, 58), ("+58", 2, 58), ("-59", 3, 59)):
        _, c, _ = derive(["--ttl=" + a])
        assert (c.ttl_mode, c.ttl_value) == (mode, val)


def test_gpu_required_without_device(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    te = TA.TcpEdit(["--fixcsum"])
    with pytest.raises(RuntimeError, match="no HIP device"):
        TA.Batch(te, open(os.path.join(ROOT, "tests", "golden", "test.pcap"), "rb").read())


def test_fuzz_options_reach_the_device_config(built):
    import oracle_lib as O
    _, c, _ = derive(["--fuzz-seed=42", "--fuzz-factor=2"])
    assert c.fuzz_seed == O.mix_seed(42) and c.fuzz_factor == 2
    _, c, _ = derive(["--fuzz-seed=42"])  # fuzz-factor defaults to 8 (tcpedit_opts.def:324-330)
    assert c.fuzz_seed == O.mix_seed(42) and c.fuzz_factor == 8
    _, c, _ = derive(["--fixcsum"])
    assert c.fuzz_seed == 0
    for bad in (["--fuzz-factor=2"], ["--fuzz-seed=1", "--fuzz-factor=0"]):
        with pytest.raises(ValueError):
            derive(bad)


def test_wave_tile_budgets_per_config_and_batch(built):
    """the wave lane's tile budget for a config and a batch (te_wave_tile_bytes: the instance
    wave_pick takes): a seed-only config runs the lean SEED instance (--seed's rewrite_ip
    without a map changes nothing, edit_packet.c:787-878); batches of small records (the
    TE_FF_SMALL mode) keep 5 KiB tiles on the lean instances and 6 KiB on the cfg-reading
    ones; the others cut 8 KiB (round 6).  Host logic only: no kernel runs."""
    L = ctypes.CDLL(TA.LIB_PATH)
    f = L.te_wave_tile_bytes
    f.restype, f.argtypes = ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    NONE, GROW, VDEL, EFCS, MTU, FUZZ = 0, 1, 2, 3, 4, 5
    pnat = "--pnat=10.0.0.0/8:192.168.0.0/16"
    cases = [
        (["--seed=42", "--fixcsum"], NONE, 1, 5120), (["--seed=42", "--fixcsum"], NONE, 0, 8192),
        (["--seed=42"], NONE, 1, 5120), (["--fixcsum"], NONE, 1, 5120), (["--fixcsum"], NONE, 0, 8192),
        ([pnat, "--fixcsum"], NONE, 0, 8192), ([pnat, "--fixcsum"], NONE, 1, 6144),
        ([pnat, "--seed=7", "--fixcsum"], NONE, 1, 6144),
        (["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"], GROW, 0, 9216),
        (["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"], GROW, 1, 9216),
        (["--enet-vlan=del", "--fixcsum"], VDEL, 1, 9216), (["--efcs", "--fixcsum"], EFCS, 0, 9216),
        (["--mtu=1000", "--mtu-trunc", "--fixcsum"], MTU, 1, 9216),
        (["--fuzz-seed=42", "--fuzz-factor=2"], FUZZ, 0, 9216),
    ]
    for args, sz, small, want in cases:
        te, cfg, _ = derive(args)
        try:
            assert f(ctypes.addressof(cfg), sz, small) == want, (args, sz, small)
        finally:
            te.close()
