"""The bench's extra lines, one workload at a time (diagnostic): the first run's result
(generic-lane tiles, lane kind) and the pipeline vs kernel-only times over the same runs,
for the bench's own seed (11) and the primary line's (1)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

if os.environ.get("XP_TORCH"):  # (the bench process has torch's device context)
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")

keep = []
if os.environ.get("XP_PRIMARY"):  # (the bench's primary line first, its batch left open)
    te0, b0, _, _, _ = bench.run_workload("c2", 1_000_000, 0, 10, seed=1, device=0, verify=False)
    b0.time_kernels(int(os.environ.get("XP_PRIMARY")))
    b0.time(int(os.environ.get("XP_PRIMARY")))
    keep.append((te0, b0))
    if os.environ.get("XP_CLOSE"):
        b0.close()
        te0.close()
for wl in (sys.argv[1:] or ["vdel", "mtu", "c4", "c3"]):
    for seed in (11, 1):
        n = bench.DEFAULT_PACKETS[wl]
        te, b, r, _, _ = bench.run_workload(wl, n, 0, 3, seed=seed, device=0, verify=bool(os.environ.get("XP_VERIFY")))
        if os.environ.get("XP_WINDOWS"):  # alternating pipeline / kernel-only windows after the first run
            for i in range(int(os.environ.get("XP_WINDOWS"))):
                p = b.time(20)
                _, kk = b.time_kernels(20)
                print(f"{wl} window {i}: pipeline {p:.4f} ms, kernel {kk:.4f} ms", flush=True)
        b.time(20)
        pk, kk = b.time_kernels(20)
        p = b.time(20)
        r2 = b.result()
        print(f"{wl} seed {seed}: generic_tiles {r.generic_tiles} fast_kind {r.fast_kind} listed_after {r2.generic_tiles} "
              f"pipeline {p:.4f} ms, kernel {kk:.4f} ms (event-pair run {pk:.4f})", flush=True)
        b.close()
        te.close()
