"""A/B timing of the edit pipeline on the three single-GPU BASELINE shapes, for the
library variant selected by TCPEDIT_HIP_LIB (diagnostic, not the bench).  Each run's
output is checked against the oracle before it is timed."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

CASES = {
    "c2": (lambda: S.pcap_fixed(1_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
    "c2x10": (lambda: S.pcap_fixed(10_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
    # small records under a cfg-reading instance (address map + port map)
    "c2pnat": (lambda: S.pcap_fixed(1_000_000, 64, seed=1),
               ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]),
    "hdr": (lambda: S.pcap_imix(1_000_000, seed=1), ["--ttl=+1", "--tos=7"]),
    "c3": (lambda: S.pcap_imix(1_000_000, seed=1),
           ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]),
    "c5": (lambda: S.pcap_mixed_v4v6(250_000, 1514, seed=1), ["--fixcsum"]),
    "c4": (lambda: S.pcap_imix(1_000_000, seed=1),
           ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
            "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add", "--enet-vlan-tag=45",
            "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"]),
    "vdel": (lambda: S.pcap_imix(1_000_000, seed=1, vlan=0xB02D), ["--enet-vlan=del", "--fixcsum"]),
    "efcs": (lambda: S.pcap_imix(1_000_000, seed=1, fcs=True), ["--efcs", "--fixcsum"]),
    # generic-lane configs (size changes by record, MAC seed, fuzzing)
    "mtu": (lambda: S.pcap_imix(1_000_000, seed=1), ["--mtu=1000", "--mtu-trunc", "--fixcsum"]),
    "macseed": (lambda: S.pcap_imix(1_000_000, seed=1), ["--enet-mac-seed=42", "--fixcsum"]),
    "fz": (lambda: S.pcap_imix(1_000_000, seed=1), ["--fuzz-seed=42", "--fuzz-factor=2"]),
}
CACHES = {"c4": lambda: S.tcpprep_cache(1_000_000, seed=1)}


def main():
    tag = os.environ.get("AB_TAG", os.path.basename(TA.LIB_PATH))
    for name in (sys.argv[1:] or list(CASES)):
        gen, args = CASES[name]
        pcap = gen()
        cache = CACHES[name]() if name in CACHES else None
        _, exp = O.rewrite(pcap, args, cache)
        te = TA.TcpEdit(args)
        b = TA.Batch(te, pcap, cache)
        rc = b.run()
        r = b.result()
        ok = rc == 0 and b.output() == exp
        b.time(5)
        pipe, kern = b.time_kernels(50)
        pipe2 = b.time(200)
        ab = r.bytes_in + r.bytes_out
        print(f"{tag:28s} {name} ok={ok} kind={r.fast_kind} generic_tiles={r.generic_tiles} "
              f"kernel_us={kern * 1e3:8.1f} pipe_us={pipe2 * 1e3:8.1f} "
              f"kernel_frac={ab / (kern * 1e-3) / 8e12:.3f} pipe_frac={ab / (pipe2 * 1e-3) / 8e12:.3f}",
              flush=True)
        b.close()
        te.close()


if __name__ == "__main__":
    main()
