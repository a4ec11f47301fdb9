# wave-lane store iteration: grow / shrink / parity tests, A/B timings, stamps for C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_shrink.py tests/test_gpu_parity.py tests/test_fast_lane.py tests/test_q8.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1; rc=$?; tail -4 gpurun_out/iter_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/ab.py c2 c3 c4 c5 > gpurun_out/iter_ab.log 2>&1 || { tail -5 gpurun_out/iter_ab.log; exit 1; }
cat gpurun_out/iter_ab.log
STAMP_CASES="c4" bash tools/gpu_stamps.sh
