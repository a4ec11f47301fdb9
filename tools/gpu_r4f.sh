set -o pipefail
mkdir -p gpurun_out
# (stamps skipped)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused.py tests/test_device_index.py -m gpu > gpurun_out/r4f_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
timeout -k 10 200 python tools/fused_probe.py 200 2>&1 | grep -v amdgpu.ids
