#!/bin/bash
# lean exact-path tiles at 8 KiB: the wave-lane GPU tests, then the bench lines they touch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_fast_lane.py tests/test_gpu_parity.py tests/test_device_index.py tests/test_shrink.py tests/test_static_fallback.py tests/test_quirks.py tests/test_q8.py > gpurun_out/bigtile_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bigtile_tests.log; grep FAILED gpurun_out/bigtile_tests.log | head; [ $rc -eq 0 ] || exit $rc
AB_VARIANTS="base" AB_WLS="c5 c2 c2x10 seed c3" bash tools/gpu_abbench.sh
