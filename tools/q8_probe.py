"""Q8 diagnostics: pipelined and prefixed-batch replays whose stale bytes come from the
capture's zeroed start (no donor record anywhere)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
from test_q8 import _overstate

recs = S.records(S.pcap_fixed(30_000, 90, ipv6=True, proto=17, seed=11))
for bad in ([9_600], [10_400], [15_000]):
    pcap = S.build_pcap(_overstate(recs, bad, by=40))
    rc_o, exp = O.rewrite(pcap, ["--fixcsum"])
    te = TA.TcpEdit(["--fixcsum"])
    rc, out = te.rewrite_pipelined(pcap, chunk_bytes=1 << 20)
    print("pipelined", bad, rc, rc_o, out == exp, te.geterr() if rc else "", flush=True)
    te.close()
    for cut_at in (9_000, bad[0] - 5):
        cut = 24 + sum(16 + r[2] for r in recs[:cut_at])
        te = TA.TcpEdit(["--fixcsum"])
        b = TA.Batch(te, memoryview(pcap)[cut:], pkt_base=cut_at, hdr=pcap[:24])
        b.set_prefix(memoryview(pcap)[24:cut])
        rc = b.run()
        r = b.result()
        print("  batch cut", cut_at, rc, r.stale_records, r.unsupported, te.geterr() if rc else "", flush=True)
        b.close()
        te.close()
