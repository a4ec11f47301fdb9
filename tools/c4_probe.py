"""C4's wave-lane kernel time (diagnostic A/B): 12.5M IMIX records, the C4 options and cache"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
C4 = ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
      "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add", "--enet-vlan-tag=45",
      "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"]
n = 12_500_000
pcap = S.pcap_imix(n, seed=1)
cache = S.tcpprep_cache(n, seed=1)
te = TA.TcpEdit(C4)
b = TA.Batch(te, pcap, cache)
b.run()
r = b.result()
alg = r.bytes_in + r.bytes_out
ms = b.time(20)
ref = b.output_np()
print(f"c4 {ms:.4f} ms frac {alg / (ms * 1e-3) / 8e12:.4f}", flush=True)
import numpy as np, hashlib
print("sha", hashlib.sha256(ref.tobytes()).hexdigest()[:16])
