# round-2 new paths on the GPU: device index, pcapng, shrink, regex/unique-ip (one call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_device_index.py tests/test_pcapng.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2_tests.log 2>&1; rc=$?; tail -30 gpurun_out/r2_tests.log; exit $rc
