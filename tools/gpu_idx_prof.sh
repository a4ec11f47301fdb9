# device index: probe + rocprofv3 kernel stats (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/idx_probe.py 50 > gpurun_out/idx_probe.txt 2>&1 || { cat gpurun_out/idx_probe.txt; exit 1; }
cat gpurun_out/idx_probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_idx -o idx -- python tools/idx_probe.py 20 > gpurun_out/prof_idx.log 2>&1 || { tail -20 gpurun_out/prof_idx.log; exit 1; }
f=$(find gpurun_out/prof_idx -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
