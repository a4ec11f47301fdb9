"""Device record index probe: C2 (1M x 64 B) and IMIX batches, index_device() ms per build.
Run under rocprofv3 --kernel-trace --stats to split the index kernel from its memset."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for name, pcap in (("c2", S.pcap_fixed(1_000_000, 64, seed=1)), ("imix", S.pcap_imix(1_000_000, seed=2))):
    te = TA.TcpEdit(["--seed=42", "--fixcsum"])
    b = TA.Batch(te, pcap)
    applied, ms = b.index_device(iters=iters)
    b.run()
    print(f"{name}: {len(pcap)} bytes, applied={applied}, index ms/build={ms:.4f}", flush=True)
    b.close()
    te.close()
