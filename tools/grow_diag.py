"""VLAN-add (static +4) diagnostics: tile counts, listed tiles, status bytes and timings
per workload (diagnostic, not a test)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
import tcpreplay_amd as TA  # noqa: E402
from tcpreplay_amd import synth as S  # noqa: E402

C4 = ["--endpoints=10.10.0.1:10.10.0.2", "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
      "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16", "--enet-vlan=add", "--enet-vlan-tag=45",
      "--enet-vlan-pri=5", "--enet-vlan-cfi=1", "--fixcsum"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
for name, args, cache in (("vlan-only", ["--enet-vlan=add", "--enet-vlan-tag=45", "--fixcsum"], False),
                          ("c4", C4, True)):
    pcap = S.pcap_imix(n, seed=1)
    c = S.tcpprep_cache(n, seed=1) if cache else None
    _, exp = O.rewrite(pcap, args, c)
    te = TA.TcpEdit(args)
    b = TA.Batch(te, pcap, c)
    rc = b.run()
    r = b.result()
    ok = rc == 0 and b.output() == exp
    st = b.status()
    hist = {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    print(f"{name}: ok={ok} n_tiles={r.n_tiles} fast_lane={r.fast_lane} kind={r.fast_kind} "
          f"listed={r.generic_tiles} status_hist={hist}", flush=True)
    pipe = b.time(20)
    print(f"   pipe_us={pipe * 1e3:.1f} after-run listed={b.result().generic_tiles}", flush=True)
    b.close()
    te.close()
