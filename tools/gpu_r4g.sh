set -o pipefail
mkdir -p gpurun_out
echo "== product"; timeout -k 10 200 python tools/fused_probe.py 200 2>&1 | grep -v amdgpu.ids || exit 1
echo "== s128"; TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_s128.so timeout -k 10 200 python tools/fused_probe.py 200 2>&1 | grep -v amdgpu.ids || exit 1
TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_s128.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused.py -m gpu > gpurun_out/r4g_tests.log 2>&1 || { echo S128 TESTS FAILED; tail -20 gpurun_out/r4g_tests.log; exit 1; }
tail -1 gpurun_out/r4g_tests.log
