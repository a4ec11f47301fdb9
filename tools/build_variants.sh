#!/bin/bash
# Builds A/B variants of libtcpedit_hip.so into tcpreplay_amd/lib/var/ (diagnostics only;
# select one at run time with TCPEDIT_HIP_LIB=<path>).  Host and kernel objects are
# compiled with the same -D flags, since the host cuts tiles to the kernel's budget.
# usage: tools/build_variants.sh name "-DFLAG=.. -DFLAG=.." [name "flags"]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/tcpreplay_amd/csrc
OUT=$ROOT/tcpreplay_amd/lib/var
mkdir -p "$OUT"
INC="-I$CS/include -I$CS/kernels -I$ROOT/include -I/opt/rocm/include"
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    tmp=$(mktemp -d)
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $INC $flags -c "$CS/kernels/tcpedit_kernels.hip" -o "$tmp/k.o" &
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $INC $flags -c "$CS/kernels/te_index.hip" -o "$tmp/ix.o" &
    for f in te_args te_api te_autoopts te_pcapng; do
        gcc -O2 -std=gnu11 -fPIC -D__HIP_PLATFORM_AMD__ $INC $flags -c "$CS/host/$f.c" -o "$tmp/$f.o"
    done
    wait
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libtcpedit_hip_$name.so" "$tmp"/*.o \
        -Wl,-soname,libtcpedit_hip.so
    rm -rf "$tmp"
    echo "built $OUT/libtcpedit_hip_$name.so ($flags)"
done
