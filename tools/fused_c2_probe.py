import os, sys
sys.path.insert(0, "/root/repo")
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
pcap = S.pcap_fixed(1_000_000, 64, seed=1)
te = TA.TcpEdit(["--seed=42", "--fixcsum"])
b = TA.Batch(te, pcap)
b.run()
print("fused ms", b.time_fused(200), flush=True)
b.close(); te.close()
