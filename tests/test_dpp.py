"""The wave's DPP helpers (tcpreplay_amd/csrc/kernels/wave_dpp.hpp: wave_prev, wave_scan_add,
wave_scan_max, wave_or) on an MI355X, against the same values computed on the host and the
LDS shift they replace (tests/dpp/dpp_probe.hip, one wave), and the DPP behaviours the
product's build depends on.

- Under full EXEC (where the product calls them) the helpers are exact.  Under a divergent
  EXEC a DPP operand read from a lane EXEC has switched off returns 0 (bound_ctrl).
- A DPP op right behind an SALU write of EXEC (the join of a divergent branch) reads the new
  EXEC's lanes: no wait states are needed.
- The cause VERDICT r4 asked about (the first wk_store_mtu's wrong pass-2 bytes): the
  compiler's DPP combine had folded `q - wave_prev(my_op)` into `v_subrev_u32_dpp ...
  wave_shr:1`, and on MI355X a DPP lane pattern on a reversed VOP2 op (v_subrev, v_lshlrev)
  applies to src1, not src0.  The product builds with the combine off (Makefile)."""
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


def _run_exec(vals, part):
    lib = ctypes.CDLL(LIB)
    lib.dpp_exec_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    lib.dpp_exec_run.restype = ctypes.c_int
    v = np.asarray(vals, np.uint32)
    out = np.zeros(5 * 64, np.uint32)
    assert lib.dpp_exec_run(v.ctypes.data, part, out.ctypes.data) == 0
    return out.reshape(5, 64)


@pytest.mark.parametrize("part", [0x5555555555555555, 0xFFFF0000FFFF0000, 0x00000000FFFFFFFF, 0x8000000000000001])
def test_dpp_right_behind_an_exec_write(built, part):
    """An SALU write of EXEC directly followed by a DPP shift (the asm sequence, then a
    compiled branch join): the DPP op reads the lanes the new EXEC has on, with no wait
    states in between as with 5, and so do the product's helper and the bare builtin."""
    v = np.arange(2000, 2064, dtype=np.uint32)
    nowait, wait5, helper, bare = _run_exec(v, part)[:4]
    exp = np.concatenate([[0], v[:-1]]).astype(np.uint32)
    src_on = np.array([lane > 0 and (part >> (lane - 1)) & 1 for lane in range(64)])
    stale = np.where(src_on, exp, 0).astype(np.uint32)
    print(f"part {part:#018x}: no wait states {'== shift' if (nowait == exp).all() else '== stale EXEC' if (nowait == stale).all() else 'other'};"
          f" bare DPP behind a join {'== shift' if (bare == exp).all() else '== stale EXEC' if (bare == stale).all() else 'other'}")
    assert (wait5 == exp).all()
    assert (helper == exp).all()
    assert (nowait == exp).all()
    assert (bare == exp).all()


def _run_vop2(a):
    lib = ctypes.CDLL(LIB)
    lib.dpp_vop2_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.dpp_vop2_run.restype = ctypes.c_int
    out = np.zeros(7 * 64, np.uint32)
    assert lib.dpp_vop2_run(a.ctypes.data, out.ctypes.data) == 0
    return out.reshape(7, 64)


A = np.arange(7, 7 + 64 * 3, 3, dtype=np.uint32)
LANES = np.arange(64, dtype=np.uint64)
B = (1000000 + 1000 * LANES).astype(np.uint32)
PREV = np.concatenate([[0], A[:-1]]).astype(np.uint32)


def test_dpp_folded_into_vop2(built):
    """wave_shr:1 on src0 of v_sub / v_add / v_max / v_or (forms the compiler's DPP combine
    makes): d = prev(a) - b, prev(a) + b, max(prev(a), b), prev(a) | b"""
    subrev, sub, add, mx, subrev_row, orv, shl = _run_vop2(A)
    assert (sub == (PREV - B).astype(np.uint32)).all()
    assert (add == (PREV + B).astype(np.uint32)).all()
    assert (mx == np.maximum(PREV, B)).all()
    assert (orv == (PREV | B)).all()


def test_dpp_on_subrev_is_not_src1_minus_src0(built):
    """v_subrev_u32 with DPP (wave_shr:1 or row_shr:1) does not give b - prev(a) on MI355X but
    prev(b) - a: the lane pattern lands on src1 (and v_lshlrev_b32's likewise) -- the wrong
    output of the first wk_store_mtu, whose `q - pop` the compiler folded into
    `v_subrev_u32_dpp v2, v78, v2 wave_shr:1`.  The product builds with the DPP combine off
    (tcpreplay_amd/csrc/Makefile), so no DPP op is folded into another."""
    subrev, _, _, _, subrev_row, _, shl = _run_vop2(A)
    rowprev = np.where(LANES % 16 == 0, 0, PREV).astype(np.uint32)
    cands = {"b - prev(a)": B - PREV, "prev(a) - b": PREV - B, "b - a": B - A, "a - b": A - B, "b": B,
             "prev(b) - a": np.concatenate([[0], B[:-1]]).astype(np.uint32) - A}
    name = lambda got: [k for k, v in cands.items() if (got == v.astype(np.uint32)).all()]
    print("v_subrev_u32_dpp wave_shr:1 ->", name(subrev), subrev[:4], "; row_shr:1 ->", name(subrev_row),
          subrev_row[:4], "; v_lshlrev_b32_dpp ->", shl[:4], "(b << prev(a) & 31:",
          ((B.astype(np.uint64) << (PREV.astype(np.uint64) & 31)) & 0xFFFFFFFF).astype(np.uint32)[:4], ")")
    prevb = np.concatenate([[0], B[:-1]]).astype(np.uint32)
    rowprevb = np.where(LANES % 16 == 0, 0, prevb).astype(np.uint32)
    assert (subrev == (prevb - A).astype(np.uint32)).all()
    assert (subrev_row == (rowprevb - A).astype(np.uint32)).all()
    assert (shl == ((prevb.astype(np.uint64) << (A.astype(np.uint64) & 31)) & 0xFFFFFFFF).astype(np.uint32)).all()
