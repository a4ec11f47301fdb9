# round 2 (re-entry): GPU suite + smoke + bench, then the generic-lane occupancy A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
for v in mw3 mw2 mw2s56; do
  TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_$v.so AB_TAG=$v timeout -k 10 300 python -u tools/ab.py mtu macseed fz c2 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  cat gpurun_out/ab_$v.log
done
