"""Device-resident timing of the tcpprep classification kernel (tp_classify):
records/s and algorithmic bytes/s on C2 (1M x 64B) and IMIX (10M, C3's corpus)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcpreplay_amd import synth  # noqa: E402
from tcpreplay_amd import tcpprep as TP  # noqa: E402



def main():
    out = {}
    for name, mk in (("c2_1m_64B", lambda: synth.pcap_fixed(1_000_000, 64, seed=1)),
                     ("imix_10m", lambda: synth.pcap_imix(10_000_000, seed=1))):
        t0 = time.time()
        pcap = mk()
        for mode in (["--port"], ["--cidr=10.0.0.0/9,172.16.128.0/17"], ["--auto=bridge"], ["--auto=first"]):
            tp = TP.TcpPrep(["--no-arg-comment"] + mode)
            ms, n = tp.time(pcap, iters=50)
            tp.close()
            out[f"{name} {mode[0]}"] = {"records": n, "kernel_ms": round(ms, 4), "mrec_s": round(n / ms / 1e3, 1)}
            print(name, mode, n, f"{ms:.4f} ms", f"{n / ms / 1e3:.1f} Mrec/s", flush=True)
        print("built+timed in", round(time.time() - t0, 1), "s", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
