set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_dlt_wireless.py tests/test_dlt_decoders.py "tests/test_dist.py::test_two_rank_gpu_q18_carry_crosses_the_cut" tests/test_fuzz_wave.py > gpurun_out/q18_tests.log 2>&1
rc=$?; tail -5 gpurun_out/q18_tests.log; grep -E "FAILED|Error" gpurun_out/q18_tests.log | head -20; exit $rc
