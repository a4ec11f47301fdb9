"""window mode vs the exact path, device-resident, K runs each (diagnostic): ms per run and
the fraction of HBM peak on the algorithmic bytes"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402
K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for name, gen, args in (("c2", lambda: S.pcap_fixed(1_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
                        ("c2x10", lambda: S.pcap_fixed(10_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
                        ("c3", lambda: S.pcap_imix(2_000_000, seed=1),
                         ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]),
                        ("c5", lambda: S.pcap_mixed_v4v6(250_000, 1514, seed=1), ["--fixcsum"])):
    pcap = gen()
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap)
    b.run()
    r = b.result()
    alg = r.bytes_in + r.bytes_out
    ex = b.time(K)
    applied, ims = b.index_device(iters=max(5, K // 10))
    fu = b.time_fused(K)
    ok = b.run_fused() == 0 and b.fused_fallbacks == 0
    f = lambda ms: round(alg / (ms * 1e-3) / 8e12, 4) if ms else None
    print(f"{name}: exact {ex:.4f} ms ({f(ex)}) index+exact {ims + ex:.4f} ({f(ims + ex)}) "
          f"fused {fu if fu is None else round(fu, 4)} ms ({f(fu)}) fused_ok={ok}", flush=True)
    b.close()
    te.close()
