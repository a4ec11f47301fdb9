# generic-lane checksum (dword loads in flight): A/B vs the previous build (mw3), then the
# full suite, smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TAG=new timeout -k 10 200 python -u tools/ab.py mtu fz macseed > gpurun_out/ab_new.log 2>&1 || { tail -5 gpurun_out/ab_new.log; exit 1; }
cat gpurun_out/ab_new.log
TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_mw3.so AB_TAG=old timeout -k 10 200 python -u tools/ab.py mtu fz macseed > gpurun_out/ab_old.log 2>&1 || { tail -5 gpurun_out/ab_old.log; exit 1; }
cat gpurun_out/ab_old.log
bash tools/gpu_suite.sh
