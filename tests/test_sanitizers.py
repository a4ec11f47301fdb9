"""Host code under the sanitizers (CPU only; GPU sanitizers are not available): the
library's option parsers (tcpedit, tcpprep incl. the regex DFA compiler, tcpreplay),
its record walk with the walker pool, and the CPU oracle -- built with
-fsanitize=address,undefined and with -fsanitize=thread (tests/sanitize/Makefile) and
driven over the option pool and captures here.  A sanitizer report fails the test."""
import fcntl
import os
import subprocess

import pytest

import golden_cases as G
import tcpprep_cases as T
from tcpreplay_amd import synth as S

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


def _pcapng_files(tmp):
    """pcapng images for the converter: good ones and malformed blocks (interface ids past
    the described interfaces, including ones negative as an int, captured lengths past the
    block, truncation)"""
    import struct
    import test_pcapng as N
    e = "<"
    shb = N._block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    idb = N._block(e, 1, struct.pack(e + "HHI", 1, 0, 100))
    imgs = [N.to_pcapng(G.read("test.pcap")), N.to_pcapng(G.read("test.pcap"), ">", 9, 7, "opb")]
    for ifn, cl in [(1, 60), (0x80000000, 60), (0xFFFFFFFF, 60), (0, 0xFFFFFFF0), (0, 0x7FFFFFFF), (0, 200)]:
        imgs.append(shb + idb + N._block(e, 6, struct.pack(e + "IIIII", ifn, 0, 0, cl, 60) + bytes(60)))
    imgs.append(imgs[0][:-7])
    paths = []
    for k, img in enumerate(imgs):
        p = os.path.join(tmp, f"ng{k}.pcapng")
        with open(p, "wb") as f:
            f.write(img)
        paths.append(p)
    return paths


def _cases(path, ng_paths=()):
    import test_gpu_parity as P
    lines = [["rewrite"] + a for a in P.OPTION_POOL]
    lines += [["rewrite", "--bogus"], ["rewrite", "--pnat=not-a-cidr"], ["rewrite", "--portmap=70000:1"],
              ["rewrite", "--enet-dmac=zz"], ["rewrite", "--mtu=-1", "--mtu-trunc"]]
    lines += [["prep"] + T.args(n) for n in T.CASES] + [["prep", "--regex=("], ["prep", "--cidr=300.1.1.1/8"],
                                                         ["prep", "--include=P:5-"], ["prep"]]
    lines += [["replay", "--unique-ip", "--loop=3"], ["replay", "--loop=0"], ["replay", "--unique-ip-loops=2"]]
    for r in ["96.17.211.*", "^(10|192)\\.", "[[:xdigit:]]{4}", "(a|b)*c{2,3}", "\\w", "(((((((((x)))))))))",
              "[^0-9.:]", "a{64}", "((1|2)+3?)*$"]:
        for s_ in ["96.17.211.1", "::ffff:1.2.3.4", "2001:db8::1", "0.0.0.0", ""]:
            lines.append(["re", r, s_ or "1"])
    lines += [["ng", p] for p in ng_paths]
    with open(path, "w") as f:
        for ln in lines:
            f.write("\t".join(ln) + "\n")


def _captures(tmp):
    paths = [os.path.join(HERE, "golden", "test.pcap")]
    big = os.path.join(tmp, "big.pcap")  # > 8 walker stretches of 2 MiB
    with open(big, "wb") as f:
        f.write(S.pcap_imix(120_000, seed=3))
    fake = b"".join(b"\x01\0\0\0\x02\0\0\0\x0c\0\0\0\x0c\0\0\0" + bytes(range(12)) for _ in range(50))
    recs = []
    for ts, tu, cl, ln, d in S.records(S.pcap_fixed(12_000, 1_442, seed=4)):
        d = bytearray(d)
        d[42:42 + len(fake)] = fake
        recs.append((ts, tu, cl, ln, bytes(d)))
    trap = os.path.join(tmp, "trap.pcap")  # 17 MiB: the walker's stretches meet the fake chains
    with open(trap, "wb") as f:
        f.write(S.build_pcap(recs))
    cut = os.path.join(tmp, "cut.pcap")
    with open(cut, "wb") as f:
        f.write(G.read("test.pcap")[:-37])
    return paths + [big, trap, cut]


@pytest.fixture(scope="module")
def drivers(built):
    os.makedirs(os.path.join(SAN, "_build"), exist_ok=True)
    with open(os.path.join(SAN, "_build", ".lock"), "w") as lk:  # xdist workers share the tree
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            r = subprocess.run(["make", "-s", "-C", SAN], capture_output=True, text=True, timeout=900)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    assert r.returncode == 0, r.stderr[-3000:]
    return {k: os.path.join(SAN, "_build", k, "san_driver") for k in ("asan", "tsan")}


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_is_clean_under_the_sanitizers(drivers, tmp_path, kind):
    cases = str(tmp_path / "cases.tsv")
    _cases(cases, _pcapng_files(str(tmp_path)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               TCPEDIT_HIP_WALK_THREADS="8")
    if kind == "tsan":
        env["SAN_NO_ORACLE"] = "1"  # the thread-sanitizer run is about the walker pool
    r = subprocess.run([drivers[kind], cases] + _captures(str(tmp_path)), capture_output=True, text=True,
                       timeout=900, env=env)
    report = r.stdout[-2000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert bad not in r.stderr, report
    assert "records walked" in r.stdout
