# fuzz wave path: the tests, then A/B of the in-tree library against lib/abvar variants on
# the fz bench line, then the rocprofv3 kernel trace of the in-tree library's fz run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_fuzz_wave.py \
    "tests/test_gpu_parity.py::test_fuzz_matches_oracle_on_mixed_captures" > gpurun_out/fzab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fzab_tests.log; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS="base ${FZ_VARIANTS} base" AB_WLS=fz bash tools/gpu_abbench.sh || exit 1
P="python3 bench.py --workload fz --steps 20 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r05_fz -o run -- $P \
    > gpurun_out/prof_r05_fz.log 2>&1 || { echo "kernel-trace FAILED"; tail -20 gpurun_out/prof_r05_fz.log; exit 1; }
grep -h "te_\|rocclr" gpurun_out/prof_r05_fz/run_kernel_stats.csv
