"""window-mode phase stamps (TE_WK_STAMPS library; diagnostic): one fused run per workload"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
for name, pcap, args in (("c2", S.pcap_fixed(1_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
                         ("c5", S.pcap_mixed_v4v6(250_000, 1514, seed=1), ["--fixcsum"])):
    te = TA.TcpEdit(args); b = TA.Batch(te, pcap)
    print("==", name, "fused ms", b.time_fused(1), "exact ms", b.time(3), flush=True)
    b.close(); te.close()
