"""run one launch per workload with the TE_FK_STAMPS library (diagnostic)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
for name, pcap, args in (("c2", S.pcap_fixed(1_000_000, 64, seed=1), ["--seed=42", "--fixcsum"]),
                         ("c5", S.pcap_mixed_v4v6(250_000, 1514, seed=1), ["--fixcsum"]),
                         ("c3", S.pcap_imix(1_000_000, seed=1), ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"])):
    te = TA.TcpEdit(args); b = TA.Batch(te, pcap)
    b.run(); b.time(2)
    print("==", name, "kernel ms", b.time(5), flush=True)
    b.close(); te.close()
