"""the window-mode pipeline on C2 at one chunk size, a few reps (diagnostic, for a trace)"""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("TCPEDIT_HIP_PIPE_TRACE", "1")
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402
chunk = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 2 << 20
pcap = S.pcap_fixed(1_000_000, 64, seed=1)
te = TA.TcpEdit(["--seed=42", "--fixcsum"])
pin_in = TA.PinnedBuffer(len(pcap))
pin_in.view[:] = pcap
pin_out = TA.PinnedBuffer(te.output_bound(pcap))
for _ in range(4):
    t0 = time.perf_counter()
    rc, v = te.rewrite_pipelined(pin_in.view, chunk_bytes=chunk, out=pin_out.view)
    print("rc", rc, "ms", round((time.perf_counter() - t0) * 1e3, 3), flush=True)
