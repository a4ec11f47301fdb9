# round 4: window mode with prefetch (occupancy A/B), the window pipeline's ramps, tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused.py tests/test_device_index.py -m gpu > gpurun_out/r4c_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
echo "== product"; timeout -k 10 200 python tools/fused_probe.py 200 2>&1 | grep -v amdgpu.ids || exit 1
echo "== win3"; TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_win3.so timeout -k 10 200 python tools/fused_probe.py 200 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/e2e_win_ab.sh 2,4,8,16 > gpurun_out/e2e_win_ab_r4c.txt 2>&1 || { echo E2E FAILED; tail -5 gpurun_out/e2e_win_ab_r4c.txt; exit 1; }
cat gpurun_out/e2e_win_ab_r4c.txt
