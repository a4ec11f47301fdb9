set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tcpprep_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/prep_tests.log 2>&1; rc=$?; tail -5 gpurun_out/prep_tests.log; exit $rc
