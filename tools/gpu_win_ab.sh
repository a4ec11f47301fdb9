#!/bin/bash
# window mode A/B (diagnostic): tools/fused_probe.py under the in-tree library ("base") and the
# variants named in WIN_VARIANTS (tcpreplay_amd/lib/abvar/libtcpedit_hip_<name>.so), in turn
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base ${WIN_VARIANTS}; do
  if [ "$v" = base ]; then L=tcpreplay_amd/lib/libtcpedit_hip.so; else L=tcpreplay_amd/lib/abvar/libtcpedit_hip_$v.so; fi
  echo "== $v"
  TCPEDIT_HIP_LIB=$L timeout -k 10 300 python3 tools/fused_probe.py ${WIN_K:-200} 2>&1 | tee gpurun_out/winab_$v.log || exit 1
done
