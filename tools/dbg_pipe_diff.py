"""GPU debugging aid: where the pipelined rewrite of one decoder/option case differs
from the oracle (first differing records, their lengths and byte diffs)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import oracle_lib as O
import tcpreplay_amd as TA
from tcpreplay_amd import synth as S
import test_dlt_decoders as D

kind, k = sys.argv[1], int(sys.argv[2])
args = D.ARGSETS[k]
pcap = S.reframe(D._base(3000, seed=k + 1), kind, odd_every=11)
rc_o, exp = O.rewrite(pcap, args)
er = S.records(exp)
for chunk in (1 << 16, 1 << 18, 1 << 20):
    te = TA.TcpEdit(args, dlt=D.DLT_OF[kind])
    rc, out = te.rewrite_pipelined(pcap, None, chunk_bytes=chunk)
    rc2, out2 = te.rewrite(pcap)
    te.close()
    gr = S.records(out)
    bad = [i for i, (a, b) in enumerate(zip(gr, er)) if a != b]
    print(f"chunk {chunk}: rc {rc}/{rc_o} recs {len(gr)}/{len(er)} batch_ok {out2 == exp} ndiff {len(bad)} first {bad[:12]}")
    for i in bad[:3]:
        a, b = gr[i], er[i]
        print("  rec", i, "gpu hdr", a[:4], "oracle hdr", b[:4])
        d = [j for j in range(min(len(a[4]), len(b[4]))) if a[4][j] != b[4][j]]
        print("  byte diffs at", d[:20], "gpu", a[4][:40].hex(), "\n  oracle", b[4][:40].hex())
