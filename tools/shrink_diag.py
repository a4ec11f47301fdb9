"""diagnostics: one --efcs case on the device lanes (default, generic only, scan placement)
and the same records without the FCS, first differing byte against the oracle"""
import os
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import fl_cases as F  # noqa: E402
import oracle_lib as O  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402
from test_shrink import fcs  # noqa: E402


def go(pcap, args, env):
    for k, v in env.items():
        os.environ[k] = v
    try:
        te = TA.TcpEdit(args)
        b = TA.Batch(te, pcap)
        rc = b.run()
        out, r = b.output(), b.result()
        b.close()
        te.close()
    finally:
        for k in env:
            del os.environ[k]
    _, exp = O.rewrite(pcap, args)
    d = next((i for i in range(min(len(out), len(exp))) if out[i] != exp[i]), None)
    print(args, env, "rc", rc, "fast", r.fast_lane, r.fast_kind, "gen", r.generic_tiles, "of", r.n_tiles, "diff", d,
          out[d - 2:d + 4].hex() if d else "", exp[d - 2:d + 4].hex() if d else "", flush=True)


base = F.mixed(3000, seed=400, near_miss=0.0)
p1 = F.build(fcs(base))
for env in ({}, {"TCPEDIT_HIP_NO_FAST": "1"}, {"TCPEDIT_HIP_NO_GROW": "1"}):
    go(p1, ["--efcs", "--fixcsum"], env)
go(F.build(base), ["--fixcsum"], {})
go(F.build(base[970:990]), ["--fixcsum"], {})
go(F.build(fcs(base[970:990])), ["--efcs", "--fixcsum"], {})

# the zero-sum record alone, and with its checksum field disturbed: is the field recomputed?
import struct  # noqa: E402
r = base[978]
d = bytearray(r[4])
d[60:62] = b"\x12\x34"
alt = (r[0], r[1], r[2], r[3], bytes(d))
for recs in ([r], [alt], base[976:980], [base[977], alt]):
    go(F.build(fcs(recs)), ["--efcs", "--fixcsum"], {})
    go(F.build(recs), ["--fixcsum"], {})
