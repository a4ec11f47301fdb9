# A/B of library variants on the ab.py cases (diagnostic)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${AB_VARIANTS:-nomix}; do
  TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_$v.so AB_TAG=$v timeout -k 10 200 python tools/ab.py ${AB_CASES:-c4} > gpurun_out/ab_$v.log 2>&1 || { tail -3 gpurun_out/ab_$v.log; }
  cat gpurun_out/ab_$v.log
done
timeout -k 10 200 python tools/ab.py ${AB_CASES:-c4}
