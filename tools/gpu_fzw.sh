# the --fuzz-seed wave path and the DPP hazard probe on the GPU, then the fz bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread -s \
    tests/test_dpp.py tests/test_fuzz_wave.py tests/test_mtu_wave.py tests/test_fast_lane.py tests/test_shrink.py "tests/test_gpu_parity.py::test_fuzz_matches_oracle_on_mixed_captures" \
    "tests/test_gpu_parity.py::test_fuzz_state_runs_across_a_million_records" \
    "tests/test_gpu_parity.py::test_fuzz_through_the_per_packet_api" > gpurun_out/fzw_tests.log 2>&1
rc=$?
tail -25 gpurun_out/fzw_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --extra fz,mtu,c3 --no-cpu-baseline --no-e2e --no-device-index \
    --no-packet-latency > gpurun_out/fzw_bench.log 2>&1
rc=$?
tail -5 gpurun_out/fzw_bench.log
exit $rc
