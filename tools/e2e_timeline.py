"""The window-mode pipeline's per-chunk timeline on C2 (diagnostic): upload, edit and
download times of every chunk relative to the first upload (TCPEDIT_HIP_PIPE_TIMELINE),
from page-locked buffers, at the chunk sizes given (MiB, default the library's)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

pcap = S.pcap_fixed(1_000_000, 64, seed=1)
te = TA.TcpEdit(["--seed=42", "--fixcsum"])
rc, ref = te.rewrite_pipelined(pcap)
ref = bytes(ref)
bi, bo = TA.PinnedBuffer(len(pcap)), TA.PinnedBuffer(te.output_bound(pcap))
bi.view[:] = pcap
for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"]):
    if len(sys.argv) > 2:
        os.environ["TCPEDIT_HIP_PIPE_ALIGN"] = sys.argv[2]
    for r in range(6):
        if r == 5:
            os.environ["TCPEDIT_HIP_PIPE_TIMELINE"] = "1"
        t0 = time.perf_counter()
        rc, v = te.rewrite_pipelined(bi.view, chunk_bytes=int(c) << 20, out=bo.view)
        el = time.perf_counter() - t0
        os.environ.pop("TCPEDIT_HIP_PIPE_TIMELINE", None)
        assert rc == 0 and bytes(v) == ref
        print(f"chunk {c} MiB run {r}: {el * 1e3:.3f} ms", file=sys.stderr, flush=True)
bi.close()
bo.close()
te.close()
