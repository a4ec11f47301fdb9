"""What slows the pipelined C2 run inside bench.py (diagnostic): the same 5 runs from
page-locked buffers after (a) nothing, (b) torch's CUDA init, (c) a C4-sized batch opened,
run and closed first (4.6 GB host capture), (d) both."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
mode = sys.argv[1]
if "torch" in mode:
    import torch
    torch.cuda.set_device(0)
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

if "big" in mode:
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
bi, bo = TA.PinnedBuffer(len(pcap)), TA.PinnedBuffer(te.output_bound(pcap))
bi.view[:] = pcap
ts = []
for r in range(9):
    t0 = time.perf_counter()
    rc, v = te.rewrite_pipelined(bi.view, out=bo.view)
    ts.append(time.perf_counter() - t0)
print(mode, " ".join(f"{t * 1e3:.3f}" for t in ts), "median", f"{sorted(ts)[4] * 1e3:.3f}", flush=True)
