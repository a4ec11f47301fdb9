set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${STAMP_CASES:-c2 c3 c4}; do
AB_TAG=stamps TCPEDIT_HIP_LIB=tcpreplay_amd/lib/var/libtcpedit_hip_stamps.so timeout -k 10 200 python tools/ab.py $c > gpurun_out/stamps_$c.log 2>&1 || { tail -5 gpurun_out/stamps_$c.log; exit 1; }
echo "== $c"; grep wstamps gpurun_out/stamps_$c.log | tail -4
grep " ok=" gpurun_out/stamps_$c.log
done
