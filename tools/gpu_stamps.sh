set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=stamps TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_stamps.so timeout -k 10 200 python tools/ab.py c2 > gpurun_out/stamps.log 2>&1 || { tail -5 gpurun_out/stamps.log; exit 1; }
grep wstamps gpurun_out/stamps.log | tail -8
grep "c2 ok" gpurun_out/stamps.log
