#!/bin/bash
# fast-lane bring-up: its parity tests first, then the whole GPU suite, then timings (A/B variants)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_fast_lane.py -x -q > gpurun_out/fast_tests.log 2>&1
rc=$?; tail -15 gpurun_out/fast_tests.log; echo "FAST EXIT $rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "not full_size" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; echo "GPU EXIT $rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
for v in b256t16p3 b128t12p3 b256t24p3 b256t32p3 b128t8p3 b256t16n4 b128t12n4; do
  if [ $v = default ]; then unset TCPEDIT_HIP_LIB TCPEDIT_HIP_NO_FAST
  elif [ $v = nofast ]; then unset TCPEDIT_HIP_LIB; export TCPEDIT_HIP_NO_FAST=1
  else export TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_$v.so; unset TCPEDIT_HIP_NO_FAST; fi
  echo "== $v"
  timeout -k 10 300 python tools/perf_matrix.py > gpurun_out/perf_$v.txt 2>&1 || { tail -5 gpurun_out/perf_$v.txt; exit 1; }
  grep -E "seed=42 --fixcsum|^1514B_mixed  --fixcsum|^imix.*pnat" gpurun_out/perf_$v.txt
done
unset TCPEDIT_HIP_LIB TCPEDIT_HIP_NO_FAST
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_fast -o run -- python3 bench.py --workload c2 --steps 20 --warmup 2 --extra= --no-cpu-baseline > gpurun_out/prof_fast.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/prof_fast.log; exit 1; }
cat gpurun_out/prof_fast/run_kernel_stats.csv
echo DONE
