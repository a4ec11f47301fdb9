"""Per-batch spread of the edit kernel's time within one process (diagnostic): the same
workload opened AP_N times (AP_KEEP: earlier batches left open, so each lands elsewhere in
HBM), kernel-only time of each over AP_ITERS runs."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "hdr"
keep = []
for i in range(int(os.environ.get("AP_N", "8"))):
    te, b, r, _, _ = bench.run_workload(wl, bench.DEFAULT_PACKETS[wl], 0, 3, seed=11, device=0, verify=False)
    b.time(20)
    ks = [b.time_kernels(int(os.environ.get("AP_ITERS", "50")))[1] for _ in range(3)]
    ab = r.bytes_in + r.bytes_out
    print(f"{wl} batch {i}: kernel ms " + " ".join(f"{k:.4f}" for k in ks) +
          f"  frac {ab / (min(ks) * 1e-3) / 8e12:.4f}", flush=True)
    if os.environ.get("AP_KEEP"):
        keep.append((te, b))
    else:
        b.close()
        te.close()
