#!/bin/bash
# GPU tests, timing matrix (default + variants) and SQ instruction-mix counters of the C2 launch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "not full_size" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; echo "GPU EXIT $rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
fi
for v in default ${VARIANTS}; do
  if [ $v = default ]; then unset TCPEDIT_HIP_LIB; else export TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_$v.so; fi
  [ $v = default ] || [ -f "$TCPEDIT_HIP_LIB" ] || { echo "skip $v"; continue; }
  echo "== $v"
  timeout -k 10 300 python tools/perf_matrix.py ${SHAPES} > gpurun_out/perf_$v.txt 2>&1 || { tail -5 gpurun_out/perf_$v.txt; exit 1; }
  grep -E "seed=42 --fixcsum|^1514B_mixed  --fixcsum|^imix.*pnat|^64B_udp4  +rc" gpurun_out/perf_$v.txt
done
unset TCPEDIT_HIP_LIB
P="python3 bench.py --workload ${WL:-c2} --steps 10 --warmup 1 --extra= --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_sq0 -o run -- $P > gpurun_out/prof_sq0.log 2>&1 && cat gpurun_out/prof_sq0/run_kernel_stats.csv
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d gpurun_out/pmc_sq -o run -- $P > gpurun_out/pmc_sq.log 2>&1 || { echo "SQ pmc failed"; tail -5 gpurun_out/pmc_sq.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA \
  --output-format csv -d gpurun_out/pmc_sq2 -o run -- $P > gpurun_out/pmc_sq2.log 2>&1 || { echo "SQ2 pmc failed"; tail -5 gpurun_out/pmc_sq2.log; }
echo DONE
