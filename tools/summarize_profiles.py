"""Copy the rocprofv3 summaries of one gpurun call into profiles/ and derive the
per-launch HBM traffic of the edit kernel from the two PMC passes.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports
half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section), so it
is doubled; WRITE_SIZE is exact for 16-byte streaming stores.

usage: python tools/summarize_profiles.py ROUND WORKLOAD [alg_bytes_per_launch]
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
KERNEL = None  # the kernel with the largest total time in the trace stats


def dominant_kernel(stats):
    rows = [r for r in csv.DictReader(open(stats)) if r["Name"].startswith("te_")]
    return max(rows, key=lambda r: float(r["TotalDurationNs"]))["Name"]


def counter(path, name):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]


def main():
    rnd, wl = sys.argv[1], sys.argv[2]
    alg = int(sys.argv[3]) if len(sys.argv) > 3 else None
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    global KERNEL
    stats = os.path.join(src, f"prof_{rnd}_{wl}", "run_kernel_stats.csv")
    KERNEL = dominant_kernel(stats)
    shutil.copy(stats, os.path.join(dst, f"{rnd}_{wl}_kernel_stats.csv"))
    fetch = counter(os.path.join(src, f"pmc_fetch_{rnd}_{wl}", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter(os.path.join(src, f"pmc_write_{rnd}_{wl}", "run_counter_collection.csv"), "WRITE_SIZE")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    traffic = int(round((2 * f_kib + w_kib) * 1024))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if r["Name"] == KERNEL:
            avg_ns = float(r["AverageNs"])
    tj_path = os.path.join(dst, "traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    tj[wl] = {"round": rnd, "kernel": KERNEL, "dispatches": len(fetch),
              "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib,
              "fetch_correction": "x2 (gfx950 FETCH_SIZE counts half of wide streaming reads)",
              "hbm_bytes_per_launch": traffic, "alg_bytes_per_launch": alg,
              "kernel_avg_ns_kernel_trace": avg_ns}
    json.dump(tj, open(tj_path, "w"), indent=1)
    print(json.dumps(tj[wl]))


if __name__ == "__main__":
    main()
