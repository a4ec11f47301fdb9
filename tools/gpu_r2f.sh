# generic-lane span load in one batch (K=10) A/B, then rocprof evidence for C2 and mtu
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base k10 base k10; do
  if [ $v = base ]; then L=; else L=tcpreplay_amd/lib/var/libtcpedit_hip_$v.so; fi
  TCPEDIT_HIP_LIB=$L AB_TAG=$v timeout -k 10 200 python -u tools/ab.py mtu macseed fz > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  cat gpurun_out/ab_$v.log
done
ROUND=r02b WLS="c2 mtu" bash tools/gpu_prof.sh
