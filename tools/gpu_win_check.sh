#!/bin/bash
# window-mode default change: its GPU tests, then the A/B timings (tools/gpu_win_ab.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_fused.py tests/test_device_index.py tests/test_reader.py tests/test_q8.py "tests/test_gpu_parity.py" -k "fused or window or win or pipelined or pipeline or chunk or index or reader or q8" > gpurun_out/wincheck_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wincheck_tests.log; grep -E "FAILED" gpurun_out/wincheck_tests.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_win_ab.sh
