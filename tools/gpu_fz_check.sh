# --fuzz-seed check (one gpurun call): the GPU tests that fuzz, then rocprofv3 kernel stats of
# the fz bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "fuzz or fz" \
    > gpurun_out/fz_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/fz_tests.log; exit 1; }
tail -2 gpurun_out/fz_tests.log
P="python3 bench.py --workload fz --steps 10 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_fz -o run -- $P \
    > gpurun_out/prof_fz.log 2>&1 || { echo "kernel-trace FAILED"; tail -20 gpurun_out/prof_fz.log; exit 1; }
grep -h "te_" gpurun_out/prof_fz/run_kernel_stats.csv
grep -o '"frac_hbm_peak": [0-9.]*\|"verified": [a-z]*' gpurun_out/prof_fz.log | head -4
