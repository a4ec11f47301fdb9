#!/bin/bash
# one optimisation iteration: GPU tests, timing matrix, phase stamps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "not full_size" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; echo "GPU EXIT $rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python tools/perf_matrix.py > gpurun_out/perf.txt 2>&1 || { tail -5 gpurun_out/perf.txt; exit 1; }
grep -E "seed=42 --fixcsum|^1514B_mixed  --fixcsum|^imix.*pnat" gpurun_out/perf.txt
if [ -f tcpreplay_amd/lib/var/libtcpedit_hip_stamps.so ]; then
TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_stamps.so timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.txt 2>&1 || { tail -5 gpurun_out/stamps.txt; exit 1; }
grep -E "==|block 0 " gpurun_out/stamps.txt | head -12
fi
echo DONE
