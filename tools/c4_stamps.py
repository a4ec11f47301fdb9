"""wave-lane phase stamps on C3 and C4 (TE_WK_STAMPS library; diagnostic)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
C4 = ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
      "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add", "--enet-vlan-tag=45",
      "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"]
C3 = ["--pnat=10.0.0.0/8:192.168.0.0/16", "--portmap=53:5353,80:8080", "--fixcsum"]
n = 2_000_000
pcap = S.pcap_imix(n, seed=1)
cache = S.tcpprep_cache(n, seed=1)
for name, args, c in (("c3", C3, None), ("c4", C4, cache), ("c4nocache", [a for a in C4 if not a.startswith("--endpoints")], None)):
    te = TA.TcpEdit(args); b = TA.Batch(te, pcap, c)
    b.run(); b.time(2)
    print("==", name, "kernel ms", b.time(3), flush=True)
    b.close(); te.close()
