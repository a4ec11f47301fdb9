#!/bin/bash
# diagnostics: option/shape timing matrix, counter list, SQ instruction mix of the C2 launch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/perf_matrix.py ${SHAPES} > gpurun_out/perf_matrix.txt 2>&1
rc=$?; cat gpurun_out/perf_matrix.txt; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_SQ" ] && exit 0
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || echo "counter list failed"
P="python3 bench.py --workload c2 --steps 5 --warmup 1 --extra= --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d gpurun_out/pmc_sq -o run -- $P > gpurun_out/pmc_sq.log 2>&1 || { echo "SQ pmc failed"; tail -5 gpurun_out/pmc_sq.log; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA \
  --output-format csv -d gpurun_out/pmc_sq2 -o run -- $P > gpurun_out/pmc_sq2.log 2>&1 || { echo "SQ2 pmc failed"; tail -5 gpurun_out/pmc_sq2.log; }
echo DONE
