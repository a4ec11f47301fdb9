# generic-lane checksum change: A/B vs the previous build (mw3 variant), stamps, full suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=new timeout -k 10 200 python -u tools/ab.py mtu fz macseed > gpurun_out/ab_new.log 2>&1 || { tail -5 gpurun_out/ab_new.log; exit 1; }
cat gpurun_out/ab_new.log
TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_mw3.so AB_TAG=old timeout -k 10 200 python -u tools/ab.py mtu fz macseed > gpurun_out/ab_old.log 2>&1 || { tail -5 gpurun_out/ab_old.log; exit 1; }
cat gpurun_out/ab_old.log
TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_gkst.so timeout -k 10 200 python -u tools/gk_stamps.py mtu > gpurun_out/gk_stamps2.log 2>&1 || { tail -5 gpurun_out/gk_stamps2.log; exit 1; }
grep -E "^==|GK block [0-3] " gpurun_out/gk_stamps2.log | tail -6
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit 1
