"""Dump the --mtu-trunc output of near-miss captures (diagnostics: compared with the
oracle on the CPU afterwards).  argv: output dir, record counts..."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import fl_cases as F  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402

recs = F.mixed(6000, seed=405, near_miss=0.25)
args = ["--mtu-trunc", "--mtu=600", "--fixcsum"]
for n in map(int, sys.argv[2:]):
    te = TA.TcpEdit(args)
    b = TA.Batch(te, F.build(recs[:n]))
    rc = b.run()
    r = b.result()
    print(n, "rc", rc, "fast", r.fast_lane, "generic_tiles", r.generic_tiles)
    open(os.path.join(sys.argv[1], f"mtu_{n}.bin"), "wb").write(b.output())
    b.close()
    te.close()
