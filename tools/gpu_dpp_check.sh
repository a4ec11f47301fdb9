# the MTU store's previous-record reads (diagnostic variants, WK_MTU_PREV_DPP) on the GPU
set -o pipefail
mkdir -p gpurun_out
for v in ${@:-1 2 3 4 5}; do
  echo "== variant WK_MTU_PREV_DPP=$v"
  TCPEDIT_HIP_LIB=tcpreplay_amd/lib/dppvar/libtcpedit_hip_prevdpp$v.so timeout -k 10 200 python -u -m pytest -q -m gpu --timeout 60 --timeout-method thread tests/test_mtu_wave.py > gpurun_out/mtu_v$v.log 2>&1; echo "rc=$?"; tail -4 gpurun_out/mtu_v$v.log
done
