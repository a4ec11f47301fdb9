# fuzz tests, then the fz bench line, then traces of fz / mtu / vdel / efcs with their gaps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_fuzz_wave.py \
    "tests/test_gpu_parity.py::test_fuzz_matches_oracle_on_mixed_captures" > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5b_tests.log; [ $rc -eq 0 ] || exit $rc
WLS="fz mtu vdel efcs" bash tools/gpu_gaps.sh
