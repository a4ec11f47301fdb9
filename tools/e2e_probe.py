"""End-to-end (host bytes -> host bytes) timing of the pipelined path by chunk size and
buffer kind, with the library's stage trace on stderr (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ["TCPEDIT_HIP_PIPE_TRACE"] = "1"
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

CHUNKS = [int(c) << 20 for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4 << 20, 16 << 20, 64 << 20]
CASES = (("c2", lambda: S.pcap_fixed(1_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
         ("c3_2M", lambda: S.pcap_imix(2_000_000, seed=1),
          ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]))
for name, gen, args in CASES[:int(sys.argv[2]) if len(sys.argv) > 2 else 2]:
    pcap = gen()
    te = TA.TcpEdit(args)
    rc, ref = te.rewrite_pipelined(pcap)
    pin_in = TA.PinnedBuffer(len(pcap))
    pin_in.view[:] = pcap
    bound = te.output_bound(pcap)
    pin_out = TA.PinnedBuffer(bound)
    src = bytearray(pcap)
    obuf = bytearray(bound)
    for chunk in CHUNKS:
        for kind in ("pageable", "pinned"):
            si, so = (src, obuf) if kind == "pageable" else (pin_in.view, pin_out.view)
            ts = []
            for _ in range(4):
                t0 = time.perf_counter()
                rc, v = te.rewrite_pipelined(si, chunk_bytes=chunk, out=so)
                ts.append(time.perf_counter() - t0)
            ok = rc == 0 and bytes(v) == ref
            t = sorted(ts)[1]
            print(f"{name} chunk={chunk >> 20}MiB {kind:8s} ok={ok} ms={t * 1e3:8.2f} GB/s_in={len(pcap) / t / 1e9:6.2f}",
                  flush=True)
    pin_in.close()
    pin_out.close()
    te.close()
