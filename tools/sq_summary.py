"""median per-dispatch SQ counters per kernel from gpurun_out/pmc_sq*/ (diagnostic)"""
import collections
import csv
import glob
import statistics
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_sq*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("__amd"):
            continue
        acc[(r["Kernel_Name"].split("(")[0][-30:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:32s} {c:24s} {statistics.median(v):16.0f}")
