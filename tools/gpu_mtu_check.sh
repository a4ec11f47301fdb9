# --mtu-trunc placement check (one gpurun call): the wave-lane mtu tests, then rocprofv3 kernel
# stats of the mtu bench line (the cut prefix kernels run once per batch)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mtu_wave.py -m gpu \
    > gpurun_out/mtu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/mtu_tests.log; exit 1; }
tail -2 gpurun_out/mtu_tests.log
P="python3 bench.py --workload mtu --steps 20 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_mtu2 -o run -- $P \
    > gpurun_out/prof_mtu2.log 2>&1 || { echo "kernel-trace FAILED"; tail -20 gpurun_out/prof_mtu2.log; exit 1; }
grep -h "te_" gpurun_out/prof_mtu2/run_kernel_stats.csv
grep -o '"frac_hbm_peak": [0-9.]*\|"verified": [a-z]*' gpurun_out/prof_mtu2.log | head -4
