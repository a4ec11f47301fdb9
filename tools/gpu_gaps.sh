# rocprofv3 kernel traces of bench workloads (WLS), with the per-run gap analysis
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r05}
for WL in ${WLS:-mtu vdel}; do
    P="python3 bench.py --workload $WL --steps 20 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${R}_${WL} -o run -- $P \
        > gpurun_out/prof_${R}_${WL}.log 2>&1 || { echo "kernel-trace $WL FAILED"; tail -20 gpurun_out/prof_${R}_${WL}.log; exit 1; }
    tail -1 gpurun_out/prof_${R}_${WL}.log | cut -c1-400
    python3 tools/trace_gaps.py gpurun_out/prof_${R}_${WL}/run_kernel_trace.csv
done
