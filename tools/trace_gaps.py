"""Per-run timeline of a bench workload from a rocprofv3 kernel trace: for each dispatch of
the dominant kernel, the gap since the previous dispatch on the device ended and the kernels
between them -- where a run's time outside its edit kernel goes.
usage: python tools/trace_gaps.py gpurun_out/prof_X/run_kernel_trace.csv [kernel]"""
import csv
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = sys.argv[2] if len(sys.argv) > 2 else "te_wave_tiles"
    gaps, between, durs = [], {}, []
    prev_end = None
    last_k_end = None
    for r in rows:
        s, e, n = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]
        if n.startswith(k):
            durs.append(e - s)
            if last_k_end is not None:
                gaps.append(s - last_k_end)
            last_k_end = e
        elif last_k_end is not None:
            between.setdefault(n, []).append(e - s)
        prev_end = e
    print(f"{k}: {len(durs)} dispatches, median {statistics.median(durs) / 1e3:.1f} us")
    if gaps:
        g = sorted(gaps)
        print(f"end-to-start between consecutive {k}: median {statistics.median(g) / 1e3:.1f} us, "
              f"min {g[0] / 1e3:.1f}, max {g[-1] / 1e3:.1f}")
    for n, v in sorted(between.items(), key=lambda x: -sum(x[1])):
        print(f"  between them: {n[:60]} x{len(v)} median {statistics.median(v) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
