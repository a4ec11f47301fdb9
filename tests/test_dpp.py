"""The wave's DPP helpers (tcpreplay_amd/csrc/kernels/wave_dpp.hpp: wave_prev, wave_scan_add,
wave_scan_max, wave_or) on an MI355X, against the same values computed on the host and the
LDS shift they replace (tests/dpp/dpp_probe.hip, one wave).

Under full EXEC (where the product calls them) they are exact.  Under a divergent EXEC a DPP
operand read from a lane EXEC has switched off returns 0 (bound_ctrl), not that lane's value
-- the wrong-output cause VERDICT r4 asked about: the first wk_store_mtu's pass-2 chunks read
the previous record's {rel, op} this way and took their bytes from the tile image's start
(0 + 0), so the product reads them from an LDS table and calls the helpers only in
wave-uniform control flow."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "dpp", "_build", "libdppprobe.so")

pytestmark = pytest.mark.gpu


def _run(vals, mask, divergent):
    lib = ctypes.CDLL(LIB)
    lib.dpp_probe_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    lib.dpp_probe_run.restype = ctypes.c_int
    v = np.asarray(vals, np.uint32)
    out = np.zeros(5 * 64, np.uint32)
    assert lib.dpp_probe_run(v.ctypes.data, mask, 1 if divergent else 0, out.ctypes.data) == 0
    return out.reshape(5, 64)


def _expect(v):
    prev = np.concatenate([[0], v[:-1]]).astype(np.uint32)
    add = np.cumsum(v.astype(np.uint64)).astype(np.uint32)
    mx = np.maximum.accumulate(v)
    return prev, add, mx, np.uint32(np.bitwise_or.reduce(v))


@pytest.mark.parametrize("seed", range(4))
def test_helpers_exact_under_full_exec(built, seed):
    rng = random.Random(seed)
    v = np.array([rng.randrange(1 << (12 if seed % 2 else 32)) for _ in range(64)], np.uint32)
    prev, add, mx, orv = _run(v, ~0 & (2**64 - 1), False)[:4]
    eprev, eadd, emx, eor = _expect(v)
    lds = _run(v, ~0 & (2**64 - 1), False)[4]
    assert (prev == eprev).all() and (prev == lds).all()
    assert (add == eadd).all() and (mx == emx).all() and (orv == eor).all()


@pytest.mark.parametrize("mask", [0x5555555555555555, 0xFFFF0000FFFF0000, 0x8000000000000001 | (0xF0 << 8),
                                  0xFFFFFFFFFFFFFFFE, 0x7FFFFFFFFFFFFFFF])
def test_prev_under_divergent_exec_reads_zero_from_off_lanes(built, mask):
    """an active lane whose source lane is active reads its value (the LDS shift agrees); one
    whose source lane is off reads 0 -- the LDS shift still reads the true previous value"""
    v = np.arange(1000, 1064, dtype=np.uint32)
    prev, lds = _run(v, mask, True)[[0, 4]]
    on = [(mask >> l) & 1 for l in range(64)]
    for lane in range(64):
        if not on[lane]:
            assert prev[lane] == 0xDEADBEEF
            continue
        assert lds[lane] == (v[lane - 1] if lane else 0)
        if lane and on[lane - 1]:
            assert prev[lane] == v[lane - 1], lane
        else:
            assert prev[lane] == 0, lane
