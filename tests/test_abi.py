"""The drop-in boundary as a relinked reference tool sees it.

* tests/abi/tcprewrite_abi.c makes tcprewrite.c:61-183's calls, in its order, against
  include/tcpedit.h, with the options only in its own AutoOpts option set
  (tcprewriteOptions): the library must find them there (te_autoopts.c).
* The context begins with the reference's tcpedit_t layout (tcpedit_types.h:49-61,
  91-153), so `tcpedit->fuzz_seed` / `->seed` (tcprewrite.c:103, tcpreplay.c:169,256)
  read the derived values.
* Every symbol include/tcpedit.h declares is exported.

CPU tests check the option bridge, the layouts and the symbol table (no device call);
the GPU tests run the ABI program over the reference's goldens.
"""
import ctypes
import json
import os
import re
import subprocess

import pytest

import golden_cases as G
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABI_DIR = os.path.join(ROOT, "tests", "abi")
ABI_BIN = os.path.join(ABI_DIR, "_build", "tcprewrite_abi")


@pytest.fixture(scope="module")
def abi(built):
    # one make at a time (pytest-xdist workers share the build dir: a relink while
    # another worker runs the binary fails with ETXTBSY)
    import fcntl
    os.makedirs(os.path.join(ABI_DIR, "_build"), exist_ok=True)
    with open(os.path.join(ABI_DIR, "_build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            subprocess.check_call(["make", "-s", "-C", ABI_DIR])
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return ABI_BIN


def _lib():
    import tcpreplay_amd as TA
    return TA.load()


# ---------------------------------------------------------------- symbols and layouts
def declared_functions():
    src = open(os.path.join(ROOT, "include", "tcpedit.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;]*\)\s*;", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "while")))


def test_library_exports_every_declared_symbol(built):
    L = _lib()
    names = declared_functions()
    assert len(names) > 60
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"declared in include/tcpedit.h but not exported: {missing}"
    for n in ("fuzzing_init", "tcpedit_set_encoder_dltplugin_byid", "tcpedit_en10mb_set_mac",
              "tcpedit_dlt_output_dlt", "tcpedit_dlt_l3data"):
        assert n in names


def test_autoopts_layout_matches_libopts(abi):
    """The bridge (te_autoopts.c) and the ABI program read/write libopts' descriptors at
    the offsets the reference's options.h gives (fixture from gen_autoopts_layout.sh)."""
    ref = json.load(open(os.path.join(G.GOLDEN_DIR, "autoopts_layout.json")))
    keys = ["sizeof_opt_desc", "optOccCt", "fOptState", "optArg", "optCookie", "pz_NAME", "pz_Name",
            "pOptDesc", "specOptIdx", "optCt", "apzArgs"]
    v = (ctypes.c_size_t * len(keys))()
    _lib().te_autoopts_layout(v, len(keys))
    assert dict(zip(keys, list(v))) == {k: ref[k] for k in keys}
    prog = json.loads(subprocess.check_output([abi, "--print-layout"]).decode())
    assert prog == {k: ref[k] for k in keys}
    assert (ref["OPTST_SET_MASK"], ref["OPTST_ARG_TYPE_MASK"], ref["OPARG_TYPE_NUMERIC"]) == (15, 0xF000, 5)


# tcpedit_types.h:49-61 / :91-153 on LP64 (bool 1 B, enums 4 B, COUNTER = unsigned long
# long with ENABLE_64BITS, TCPEDIT_ERRSTR_LEN 1024): offsets worked out field by field
REF_TCPEDIT_T = {
    "validated": 0, "dlt_ctx": 8, "runtime": 16, "runtime.packetnum": 16, "runtime.dlt1": 40,
    "runtime.errstr": 48, "runtime.warnstr": 1072, "skip_broadcast": 2096, "fixlen": 2100, "editdir": 2104,
    "rewrite_ip": 2108, "tcp_sequence_enable": 2112, "tcp_sequence_adjust": 2116, "fixcsum": 2120, "efcs": 2121,
    "ttl_mode": 2124, "ttl_value": 2128, "tos": 2132, "flowlabel": 2136, "tclass": 2140, "cidrmap1": 2144,
    "dstipmap": 2168, "seed": 2176, "portmap": 2184, "mtu": 2192, "mtu_truncate": 2196, "maxpacket": 2200,
    "fuzz_seed": 2204, "fuzz_factor": 2208, "fixhdrlen": 2212, "sizeof": 2216,
}


def test_context_head_is_the_reference_tcpedit_t_layout(tmp_path):
    fields = [k for k in REF_TCPEDIT_T if k != "sizeof"]
    body = "\n".join(f'    printf("%s %zu\\n", "{f}", offsetof(tcpedit_ref_t, {f}));' for f in fields)
    src = tmp_path / "lay.c"
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include \"tcpedit.h\"\nint main(void){\n" + body +
                   '\n    printf("sizeof %zu\\n", sizeof(tcpedit_ref_t));\n    return 0;\n}\n')
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-std=gnu11", "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict((a, int(b)) for a, b in (l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines()))
    assert got == REF_TCPEDIT_T


# ---------------------------------------------------------------- the option bridge (CPU)
def _bridge(abi, args):
    out = subprocess.run([abi, "--check-options"] + args, capture_output=True, timeout=60)
    assert out.returncode == 0, out.stderr.decode()
    head, cfg = out.stdout.decode().splitlines()[:2]
    return dict(kv.split("=") for kv in head.split()), bytes.fromhex(cfg)


def _store_cfg(args):
    import tcpreplay_amd as TA
    te = TA.TcpEdit(args)
    try:
        buf = ctypes.create_string_buffer(1 << 16)
        n = te._L.tcpedit_get_dev_cfg(te._ctx, buf, len(buf), None)
        return buf.raw[:n]
    finally:
        te.close()


@pytest.mark.parametrize("case", G.IN_SCOPE, ids=[c[0] for c in G.IN_SCOPE])
def test_autoopts_bridge_derives_the_same_tables(abi, case):
    """Every golden's command line, parsed into tcprewriteOptions by the program and
    read by the library through the bridge, derives the table tcpedit_parse_args does."""
    args = case[3]
    head, cfg = _bridge(abi, args)
    assert cfg == _store_cfg(args)
    assert head["validated"] == "1"


def test_context_fields_carry_the_derived_seeds(abi):
    head, _ = _bridge(abi, ["--seed=55", "--fixcsum", "--tos=7"])
    assert int(head["seed"]) == O.mix_seed(55) and head["fixcsum"] == "1" and head["tos"] == "7"
    head, _ = _bridge(abi, ["--fuzz-seed=42", "--fuzz-factor=2"])
    assert int(head["fuzz_seed"]) == O.mix_seed(42) and head["fuzz_factor"] == "2"


def test_post_args_without_an_option_source_fails_loudly(built):
    """No AutoOpts option set in the process (a ctypes host has none), no parse_args,
    no setter: tcpedit_post_args refuses instead of deriving an empty edit."""
    L = _lib()
    ctx = ctypes.c_void_p()
    assert L.tcpedit_init(ctypes.byref(ctx), 1) == 0
    try:
        assert L.tcpedit_post_args(ctx) == -1
        assert b"no option source" in L.tcpedit_geterr(ctx)
    finally:
        L.tcpedit_close(ctypes.byref(ctx))


def _setter_ctx(calls):
    L = _lib()
    ctx = ctypes.c_void_p()
    assert L.tcpedit_init(ctypes.byref(ctx), 1) == 0
    for name, *a in calls:
        f = getattr(L, name)
        f.restype = ctypes.c_int
        assert f(ctx, *a) == 0, name
    return L, ctx


def _ctx_cfg(L, ctx):
    buf = ctypes.create_string_buffer(1 << 16)
    n = L.tcpedit_get_dev_cfg(ctx, buf, len(buf), None)
    return buf.raw[:n]


SETTER_CASES = [
    ([("tcpedit_set_fixcsum", ctypes.c_bool(True)), ("tcpedit_set_ttl_mode", 2),
      ("tcpedit_set_ttl_value", ctypes.c_uint8(3)), ("tcpedit_set_tos", ctypes.c_uint8(9)),
      ("tcpedit_set_encoder_dltplugin_byname", b"enet")],
     ["--fixcsum", "--ttl=+3", "--tos=9"]),
    ([("tcpedit_en10mb_set_vlan_mode", 2), ("tcpedit_en10mb_set_vlan_tag", ctypes.c_uint16(45)),
      ("tcpedit_en10mb_set_vlan_priority", ctypes.c_uint8(5)), ("tcpedit_en10mb_set_vlan_cfi", ctypes.c_uint8(1)),
      ("tcpedit_set_encoder_dltplugin_byid", 1)],
     ["--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-cfi=1", "--enet-vlan-pri=5"]),
    ([("tcpedit_en10mb_set_mac", b"00:12:13:14:15:16", 4), ("tcpedit_en10mb_set_mac", b"00:22:33:44:55:66", 8),
      ("tcpedit_en10mb_set_mac", b"00:22:33:44:55:66", 1), ("tcpedit_en10mb_set_mac", b"00:12:13:14:15:16", 2),
      ("tcpedit_set_port_map", b"80:8080"), ("tcpedit_set_encoder_dltplugin_byid", 1)],
     ["--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66", "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16",
      "--portmap=80:8080"]),
]


@pytest.mark.parametrize("k", range(len(SETTER_CASES)))
def test_setter_api_matches_the_option_derivation(built, k):
    """tcpedit_api.h / en10mb_api.h setters (tcpedit_init, setters, encoder selection;
    no post_args, as a setter caller runs) give the table the equivalent options give."""
    calls, args = SETTER_CASES[k]
    L, ctx = _setter_ctx(calls)
    try:
        assert L.tcpedit_validate(ctx) == 0
        assert _ctx_cfg(L, ctx) == _store_cfg(args)
    finally:
        L.tcpedit_close(ctypes.byref(ctx))


def test_encoder_can_be_selected_once(built):
    L, ctx = _setter_ctx([("tcpedit_set_encoder_dltplugin_byname", b"hdlc")])
    try:
        assert L.tcpedit_set_encoder_dltplugin_byid(ctx, 1) == -1
        assert b"already selected a DLT encoder: hdlc" in L.tcpedit_geterr(ctx)
        assert L.tcpedit_set_encoder_dltplugin_byname(ctx, b"raw") == -1
    finally:
        L.tcpedit_close(ctypes.byref(ctx))


def test_dlt_accessors(built):
    import tcpreplay_amd as TA
    te = TA.TcpEdit(["--dlt=hdlc", "--hdlc-address=15", "--hdlc-control=0"])
    L = te._L
    try:
        L.tcpedit_dlt_init.restype = ctypes.c_void_p
        d = ctypes.c_void_p(L.tcpedit_dlt_init(te._ctx, 1))
        assert d.value
        assert L.tcpedit_dlt_src(d) == 1 and L.tcpedit_dlt_dst(d) == 104 and L.tcpedit_dlt_output_dlt(d) == 104
        rec = G.read("test.pcap")[24 + 16:]  # the first record's bytes
        assert L.tcpedit_dlt_l2len(d, 1, rec, 60) == 14
        assert L.tcpedit_dlt_proto(d, 1, rec, 60) == 0x0008  # htons(ETHERTYPE_IP)
        assert L.tcpedit_l3proto(te._ctx, 0, rec, 60) == 0x0800
        assert L.tcpedit_l3proto(te._ctx, 0, rec, 10) == 0xffff  # ntohs(TCPEDIT_ERROR)
    finally:
        te.close()


# ---------------------------------------------------------------- the call sequence on the GPU
@pytest.mark.gpu
@pytest.mark.parametrize("case", G.IN_SCOPE, ids=[c[0] for c in G.IN_SCOPE])
def test_relinked_tcprewrite_reproduces_the_goldens(abi, tmp_path, case):
    """tcprewrite.c's own sequence -- AutoOpts options, post_args, validate,
    fuzzing_init(tcpedit->fuzz_seed, ...), tcpedit_packet per record from one static
    buffer, check_cache, --skip-soft-errors -- through the library equals test2.*."""
    name, inp, cache, args, _ = case
    out = tmp_path / "out.pcap"
    cmd = [abi, "-i", os.path.join(G.GOLDEN_DIR, inp), "-o", str(out)] + args
    if cache:
        cmd += ["-c", os.path.join(G.GOLDEN_DIR, cache)]
    r = subprocess.run(cmd, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got, exp = out.read_bytes(), G.read(name)
    assert got == exp, f"{name}: first difference at byte {next((i for i in range(min(len(got), len(exp))) if got[i] != exp[i]), min(len(got), len(exp)))}"


def test_cidr_maps_longer_than_the_inline_list_parse(built):
    """a CIDR map is unbounded (cidr.c:380-418): the first 16 pairs inline in the config,
    the count covering all of them (the rest in the context's spill list)"""
    import cfg_struct as CS
    import tcpreplay_amd as TA
    pairs = ",".join(f"10.{i}.0.0/16:172.{16 + i % 16}.{i}.0/24" for i in range(40))
    for args, field in (([f"--srcipmap={pairs}"], "srcipmap"), ([f"--pnat={pairs}"], "cidrmap1")):
        te = TA.TcpEdit(args)
        try:
            buf = ctypes.create_string_buffer(1 << 16)
            n = te._L.tcpedit_get_dev_cfg(te._ctx, buf, len(buf), None)
            cfg = CS.DevCfg.from_buffer_copy(buf.raw[:ctypes.sizeof(CS.DevCfg)])
            assert n == ctypes.sizeof(CS.DevCfg)
            assert getattr(cfg, "n_" + field) == 40
            if field == "cidrmap1":
                assert cfg.n_cidrmap2 == 40  # one -N serves both directions
            for i in range(16):
                e = getattr(cfg, field)[i]
                assert e.frm.masklen == 16 and e.to.masklen == 24 and (e.to.network >> 16) & 0xff == i
        finally:
            te.close()

