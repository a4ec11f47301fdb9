"""Phase breakdown of the generic lane (te_edit_tiles) on the generic-lane A/B cases, for a
library built with -DTE_GK_STAMPS=1 (tools/build_variants.sh gkst "-DTE_GK_STAMPS=1";
select it with TCPEDIT_HIP_LIB).  Diagnostic only: each case runs twice, the second run's
per-block s_memtime sums (100 MHz ticks) are what to read."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import tcpreplay_amd as TA  # noqa: E402
from ab import CASES  # noqa: E402

for name in (sys.argv[1:] or ["mtu", "fz", "macseed"]):
    gen, args = CASES[name]
    pcap = gen()
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap, None)
    b.run()
    print(f"== {name} {' '.join(args)} (second run)", flush=True)
    b.run()
    b.time(1)
    r = b.result()
    print(f"== {name} packets={r.packets} generic_tiles={r.generic_tiles} kind={r.fast_kind}", flush=True)
    b.close()
    te.close()
