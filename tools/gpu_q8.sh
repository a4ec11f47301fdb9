# Q8 replay + parity + quirks + ABI on the GPU (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_q8.py tests/test_quirks.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/q8_tests.log 2>&1; rc=$?; tail -25 gpurun_out/q8_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -8 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit 1
