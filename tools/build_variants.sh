#!/bin/bash
# Builds A/B variants of libtcpedit_hip.so into tcpreplay_amd/lib/var/ (diagnostics only;
# select one at run time with TCPEDIT_HIP_LIB=<path>).  Host and kernel objects are
# compiled with the same -D flags (the host cuts tiles to the kernel's budget), through
# the product Makefile with its own object directory.
# usage: tools/build_variants.sh name "-DFLAG=.. -DFLAG=.." [name "flags"]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/tcpreplay_amd/csrc
OUT=$ROOT/tcpreplay_amd/lib/var
mkdir -p "$OUT"
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    make -s -j8 -C "$CS" OBJDIR="$CS/build/var_$name/" LIB="$OUT/libtcpedit_hip_$name.so" \
        HIPFLAGS="-O3 -gline-tables-only -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-parameter -mllvm -amdgpu-dpp-combine=false $flags" \
        CFLAGS="-O2 -g -std=gnu11 -fPIC -D__HIP_PLATFORM_AMD__ -Wno-unused-parameter $flags" \
        "$OUT/libtcpedit_hip_$name.so"
    echo "built $OUT/libtcpedit_hip_$name.so ($flags)"
done
