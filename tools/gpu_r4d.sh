set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_device_index.py tests/test_gpu_parity.py -k "pipe or window" -m gpu > gpurun_out/r4d_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4d_tests.log; exit 1; }
tail -1 gpurun_out/r4d_tests.log
bash tools/e2e_win_ab.sh 2,4,8,16 > gpurun_out/e2e_win_ab_r4d.txt 2>&1 || { echo E2E FAILED; tail -5 gpurun_out/e2e_win_ab_r4d.txt; exit 1; }
cat gpurun_out/e2e_win_ab_r4d.txt
