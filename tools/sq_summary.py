"""median per-dispatch SQ counters per kernel from gpurun_out/pmc_sq*/ (diagnostic):
python tools/sq_summary.py [dir-glob]"""
import collections
import csv
import glob
import statistics
import sys
pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq*"
acc = collections.defaultdict(list)
for d in sorted(glob.glob(pat)):
    tag = d.rstrip("/").split("pmc_sq_")[-1].rsplit("_", 1)[0]
    for f in glob.glob(d + "/run_counter_collection.csv") + glob.glob(d + "/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("__amd") or "te_wave" not in r["Kernel_Name"]:
                continue
            acc[(tag, r["Kernel_Name"].split("(")[0][-34:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (t, k, c), v in sorted(acc.items()):
    print(f"{t:12s} {k:36s} {c:24s} {statistics.median(v):16.0f}")
