set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_device_index.py tests/test_gpu_parity.py tests/test_q8.py -k "pipe or window or chunk" -m gpu > gpurun_out/r4h_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
bash tools/e2e_win_ab.sh 4,8,16 > gpurun_out/e2e_win_ab_r4h.txt 2>&1 || { echo E2E FAILED; tail -5 gpurun_out/e2e_win_ab_r4h.txt; exit 1; }
cat gpurun_out/e2e_win_ab_r4h.txt
