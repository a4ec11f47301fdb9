"""diagnostics: run the vdel wave-lane case several times, report differences against the
oracle per run (record index, offset) and the lane counters"""
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import fl_cases as F  # noqa: E402
import oracle_lib as O  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402
from test_shrink import tag, fcs  # noqa: E402


def where(out, exp):
    d = next((i for i in range(min(len(out), len(exp))) if out[i] != exp[i]), None)
    if d is None:
        return "same" if len(out) == len(exp) else f"len {len(out)} vs {len(exp)}"
    pos, i = 24, 0
    for r in S.records(exp):
        if pos + 16 + r[2] > d:
            break
        pos += 16 + r[2]
        i += 1
    ndiff = sum(1 for a, b in zip(out, exp) if a != b)
    return f"byte {d} rec {i} off {d - pos - 16} ndiff {ndiff} got {out[d:d+8].hex()} exp {exp[d:d+8].hex()}"


for name, recs, args in [
    ("vdel", tag(F.mixed(3000, seed=300, near_miss=0.0), tpids=(0x8100, 0x88A8, 0x9100)), ["--enet-vlan=del", "--fixcsum"]),
    ("efcs", fcs(F.mixed(3000, seed=400, near_miss=0.0)), ["--efcs", "--fixcsum"]),
    ("vadd", F.mixed(3000, seed=300, near_miss=0.0), ["--enet-vlan=add", "--enet-vlan-tag=5", "--fixcsum"]),
]:
    pcap = F.build(recs)
    _, exp = O.rewrite(pcap, args)
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap)
    for k in range(4):
        rc = b.run()
        r = b.result()
        print(name, k, rc, "gen", r.generic_tiles, "of", r.n_tiles, where(b.output(), exp), flush=True)
    b.close()
    te.close()
