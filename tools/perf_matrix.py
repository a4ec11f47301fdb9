"""Kernel time of the edit launch over a matrix of option sets x synthetic shapes
(device-resident, hipEvents on the launch stream).  Diagnostic, not the bench."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

SHAPES = {
    "64B_udp4": lambda: S.pcap_fixed(1_000_000, 64, seed=1),
    "1514B_mixed": lambda: S.pcap_mixed_v4v6(250_000, 1514, seed=1),
    "imix": lambda: S.pcap_imix(1_000_000, seed=1),
}
ARGSETS = [[], ["--fixcsum"], ["--seed=42"], ["--seed=42", "--fixcsum"],
           ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"],
           ["--enet-vlan=add", "--enet-vlan-tag=45", "--fixcsum"]]


def main():
    only = sys.argv[1:] or list(SHAPES)
    for shape in only:
        pcap = SHAPES[shape]()
        for args in ARGSETS:
            te = TA.TcpEdit(args)
            b = TA.Batch(te, pcap)
            rc = b.run()
            r = b.result()
            b.time(3)
            ms = b.time(20)
            gbs = (r.bytes_in + r.bytes_out) / (ms * 1e-3) / 1e9
            print(f"{shape:12s} {' '.join(args)[:60]:60s} rc={rc} ms={ms:8.4f} Mpkt/s={r.packets / ms / 1e3:9.1f} "
                  f"GB/s={gbs:7.1f} frac={gbs / 8000:.3f}", flush=True)
            b.close()
            te.close()


if __name__ == "__main__":
    main()
