#!/bin/bash
# rocprofv3 evidence for the bench workloads: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md HBM section), per workload.
# Summaries go to gpurun_out/; tools/summarize_profiles.py copies them into profiles/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
for WL in ${WLS:-c2 c3 c5}; do
    P="python3 bench.py --workload $WL --steps 20 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${R}_${WL} -o run -- $P \
        > gpurun_out/prof_${R}_${WL}.log 2>&1 || { echo "kernel-trace $WL FAILED"; tail -20 gpurun_out/prof_${R}_${WL}.log; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${R}_${WL} -o run -- $P \
        > gpurun_out/pmc_fetch_${R}_${WL}.log 2>&1 || { echo "pmc FETCH $WL FAILED"; tail -20 gpurun_out/pmc_fetch_${R}_${WL}.log; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${R}_${WL} -o run -- $P \
        > gpurun_out/pmc_write_${R}_${WL}.log 2>&1 || { echo "pmc WRITE $WL FAILED"; tail -20 gpurun_out/pmc_write_${R}_${WL}.log; exit 1; }
    grep -h "te_" gpurun_out/prof_${R}_${WL}/run_kernel_stats.csv
done
echo DONE
