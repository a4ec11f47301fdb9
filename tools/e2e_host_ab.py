"""End-to-end C2 (pipelined, host bytes -> host bytes) by host-buffer kind, interleaved
rounds (diagnostic): the library's page-locked buffers (tcpedit_host_alloc: hipHostMalloc,
default flags), hipHostMalloc non-coherent, hipHostMalloc coherent, malloc'd memory
registered once (hipHostRegister), and ordinary buffers (locked per call by the library)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]

if "torch" in sys.argv[2:]:  # torch's HIP context first, as bench.py has it
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
if "big" in sys.argv[2:]:  # a C4-sized batch first, as bench.py runs before its e2e lines
    big = S.pcap_imix(12_500_000, seed=1)
    te0 = TA.TcpEdit(["--seed=3", "--fixcsum"])
    b0 = TA.Batch(te0, big)
    b0.run()
    b0.close()
    te0.close()
    del big
pcap = S.pcap_fixed(1_000_000, 64, seed=1)
te = TA.TcpEdit(["--seed=42", "--fixcsum"])
rc, ref = te.rewrite_pipelined(pcap)
n_in, n_out = len(pcap), te.output_bound(pcap)


def hm(n, flags):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), n, flags) == 0
    return memoryview((ctypes.c_char * n).from_address(p.value)).cast("B")


def reg(n):
    a = np.empty(n + 4096, np.uint8)
    off = (-a.ctypes.data) % 4096
    v = a[off:off + n]
    assert hip.hipHostRegister(v.ctypes.data, n, 0) == 0
    return v, memoryview(v).cast("B")


keep = []
kinds = {}
pb = (TA.PinnedBuffer(n_in), TA.PinnedBuffer(n_out))
keep.append(pb)
kinds["lib"] = (pb[0].view, pb[1].view)
kinds["noncoh"] = (hm(n_in, 0x80000000), hm(n_out, 0x80000000))
kinds["coh"] = (hm(n_in, 0x40000000), hm(n_out, 0x40000000))
ri, ro = reg(n_in), reg(n_out)
keep += [ri, ro]
kinds["reg"] = (ri[1], ro[1])
kinds["pageable"] = (memoryview(bytearray(n_in)), memoryview(bytearray(n_out)))
for k, (bi, bo) in kinds.items():
    bi[:] = pcap
res = {k: [] for k in kinds}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for k, (bi, bo) in kinds.items():
        ts = []
        for r in range(9):
            t0 = time.perf_counter()
            rc, v = te.rewrite_pipelined(bi, out=bo)
            ts.append(time.perf_counter() - t0)
        assert rc == 0 and bytes(v) == ref
        res[k].append(sorted(ts)[4] * 1e3)
    print("round", rnd, " ".join(f"{k} {res[k][-1]:.3f}" for k in kinds), flush=True)
print("medians", " ".join(f"{k} {sorted(v)[len(v) // 2]:.3f}" for k, v in res.items()), flush=True)
