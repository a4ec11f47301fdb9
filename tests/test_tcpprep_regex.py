"""tcpprep --regex (src/tcpprep.c:300-335): the host-compiled DFA the classifier walks
on the device (tp_regex.c) against the C library's regexec, on the strings inet_ntop
prints -- the reference's exact inputs -- for IPv4 and IPv6 sources of every shape.

CPU only: the DFA is compiled and walked on the host here (tcpprep_regex_dfa_match);
the device walk is checked against the oracle in test_tcpprep_gpu.py."""
import ctypes
import random
import socket

import pytest

import tcpreplay_amd as TA

REG_EXTENDED, REG_NOSUB = 1, 8

PATTERNS = [
    "96.17.211.*", r"^10\.", r"\.1$", r"^(10|192)\.", "[0-9]{3}", "^2001:db8::", "::ffff:", "1|2",
    "^$", "1+2?3*", "[^0-9.]", "[[:xdigit:]]{4}", "(1|12)(2|23)$", r"^[0-9]+\.[0-9]+\.[0-9]+\.[0-9]+$", ".*",
    "(ab|cd)*e", "f{2,3}", "^:", "[.]", "0{1,}", "(^1|2$)", "^::", "::$", "[a-f][0-9]:", r"^[0-9]{1,3}(\.[0-9]{1,3}){3}$",
    "^(fe80|ff0[0-9a-f]):", "([0-9a-f]{1,4}:){7}[0-9a-f]{1,4}", r"\.(25[0-5]|2[0-4][0-9])$", "^1?9?2", "x|^1",
    "[[:digit:]]+[[:punct:]]", "(0|00|000)+", "a{0}b", "^[^:]*$",
]


def _libc():
    c = ctypes.CDLL("libc.so.6")
    c.regcomp.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
    c.regexec.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    c.regfree.argtypes = [ctypes.c_void_p]
    return c


def _addresses(n, seed):
    rng = random.Random(seed)
    out = ["0.0.0.0", "255.255.255.255", "96.17.211.1", "::", "::1", "::ffff:1.2.3.4", "::1.2.3.4", "1::", "1:0:0:2::3"]
    for i in range(n):
        k = i % 6
        if k == 0:
            out.append(socket.inet_ntop(socket.AF_INET, bytes(rng.randrange(256) for _ in range(4))))
        elif k == 1:
            out.append(socket.inet_ntop(socket.AF_INET, bytes(rng.choice([0, 1, 9, 10, 96, 192, 211, 255]) for _ in range(4))))
        else:
            w = [rng.choice([0, 0, 0, rng.randrange(65536), rng.randrange(16), 0xffff]) for _ in range(8)]
            if k == 5:
                w[:6] = [0, 0, 0, 0, 0, rng.choice([0, 0xffff])]
            out.append(socket.inet_ntop(socket.AF_INET6, b"".join(x.to_bytes(2, "big") for x in w)))
    return out


@pytest.mark.parametrize("pattern", PATTERNS)
def test_dfa_agrees_with_regexec(built, pattern):
    L = ctypes.CDLL(TA.LIB_PATH)
    L.tcpprep_regex_dfa_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    c = _libc()
    rx = ctypes.create_string_buffer(256)
    assert c.regcomp(rx, pattern.encode(), REG_EXTENDED | REG_NOSUB) == 0
    try:
        for s in _addresses(3000, seed=len(pattern)):
            want = 1 if c.regexec(rx, s.encode(), 0, None, 0) == 0 else 0
            got = L.tcpprep_regex_dfa_match(pattern.encode(), s.encode())
            assert got == want, (pattern, s)
    finally:
        c.regfree(rx)


def test_unsupported_and_invalid_patterns_are_refused(built):
    """back-references and GNU escapes are refused (-1), never approximated; the tool's
    option parser reports regcomp's own error for an invalid pattern"""
    L = ctypes.CDLL(TA.LIB_PATH)
    L.tcpprep_regex_dfa_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    for p in [r"(1)\1", r"\w", r"\b1", "[[=a=]]", "(1"]:
        assert L.tcpprep_regex_dfa_match(p.encode(), b"1.1.1.1") == -1, p
    from tcpreplay_amd import tcpprep as TP
    with pytest.raises(Exception, match="regex"):
        TP.TcpPrep(["--regex=(1"])
