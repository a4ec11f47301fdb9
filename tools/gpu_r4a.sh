# round 4: window-mode stamps and timing, the new tests, e2e A/B (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
# (stamps: run separately with a fresh stamps variant)
timeout -k 10 200 python tools/win_stamps.py > gpurun_out/win_pre.txt 2>&1 || { echo PRE FAILED; tail -5 gpurun_out/win_pre.txt; exit 1; }
grep "==" gpurun_out/win_pre.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused.py tests/test_device_index.py tests/test_dlt_wireless.py tests/test_dist.py -m gpu > gpurun_out/r4a_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -2 gpurun_out/r4a_tests.log
bash tools/e2e_ab.sh 2,4,8 > gpurun_out/e2e_ab_r4.txt 2>&1 || { echo E2E FAILED; tail -5 gpurun_out/e2e_ab_r4.txt; exit 1; }
cat gpurun_out/e2e_ab_r4.txt
