# A/B of the mtu bench line: product library vs a variant (argument: variant name), twice each
# (the variant is built by tools/build_variants.sh; lift the ./tcpreplay_amd/lib/var line of .gpurunignore for the call)
set -o pipefail
mkdir -p gpurun_out
V=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_$1.so
B="python bench.py --workload mtu --steps 50 --warmup 5 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
for i in 1 2; do
    timeout -k 10 200 $B 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ' || exit 1; echo " product"
    TCPEDIT_HIP_LIB=$V timeout -k 10 200 $B 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"frac": [0-9.]*' | tr '\n' ' ' || exit 1; echo " $1"
done
