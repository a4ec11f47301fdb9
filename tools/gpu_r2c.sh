# round 2 (re-entry): device-index tests, generic-lane stamps + occupancy A/B, then the
# full GPU suite, smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_device_index.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/dix_tests.log 2>&1; rc=$?; tail -3 gpurun_out/dix_tests.log; [ $rc = 0 ] || exit 1
TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_gkst.so timeout -k 10 200 python -u tools/gk_stamps.py mtu fz macseed > gpurun_out/gk_stamps.log 2>&1 || { tail -5 gpurun_out/gk_stamps.log; exit 1; }
grep -E "^==|GK block [0-3] " gpurun_out/gk_stamps.log | tail -40
for v in mw3 mw2; do
  TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_$v.so AB_TAG=$v timeout -k 10 200 python -u tools/ab.py mtu fz > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  cat gpurun_out/ab_$v.log
done
bash tools/gpu_suite.sh
