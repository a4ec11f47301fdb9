# regex / unique-ip / tcpprep GPU tests (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_unique_ip.py tests/test_tcpprep_gpu.py tests/test_tcpprep_regex.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1; rc=$?; tail -15 gpurun_out/f_tests.log; exit $rc
