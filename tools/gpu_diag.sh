#!/bin/bash
# diagnostics for the wave lane: per-phase stamps (diagnostic build) and SQ counters
# of the C2 launch.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tcpreplay_amd/lib/var
if [ -f "$V/libtcpedit_hip_wstamps.so" ]; then
    TCPEDIT_HIP_LIB=$V/libtcpedit_hip_wstamps.so timeout -k 10 120 python -u tools/stamps.py > gpurun_out/wstamps.txt 2>&1
    rc=$?; grep "==" gpurun_out/wstamps.txt; [ $rc -eq 0 ] || { tail -5 gpurun_out/wstamps.txt; exit $rc; }
fi
[ -n "$NO_SQ" ] && exit 0
P="python3 bench.py --workload ${WL:-c2} --steps 5 --warmup 1 --extra= --no-cpu-baseline --no-e2e"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d gpurun_out/pmc_sq -o run -- $P > gpurun_out/pmc_sq.log 2>&1 || { echo "SQ pmc failed"; tail -5 gpurun_out/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA \
  --output-format csv -d gpurun_out/pmc_sq2 -o run -- $P > gpurun_out/pmc_sq2.log 2>&1 || { echo "SQ2 pmc failed"; tail -5 gpurun_out/pmc_sq2.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/pmc_sq/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv te_wave_tiles || true
echo DONE
