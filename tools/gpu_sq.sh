#!/bin/bash
# SQ counters of the wave-lane kernel per bench workload (diagnostic): two --pmc passes per
# workload and library (SQ_VARIANTS: names under tcpreplay_amd/lib/abvar; "base" = in-tree)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--steps 20 --warmup 2 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency --no-verify"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for v in ${SQ_VARIANTS:-base}; do
  if [ "$v" = base ]; then L=tcpreplay_amd/lib/libtcpedit_hip.so; else L=tcpreplay_amd/lib/abvar/libtcpedit_hip_$v.so; fi
  for w in ${WLS:-c2}; do
    i=0
    for P in "$P1" "$P2"; do
      i=$((i+1))
      TCPEDIT_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_sq_${v}_${w}_$i -o run -- python3 bench.py --workload $w $F > gpurun_out/pmc_sq_${v}_${w}_$i.log 2>&1 || { echo "pmc $v $w $i FAILED"; tail -5 gpurun_out/pmc_sq_${v}_${w}_$i.log; exit 1; }
    done
    echo "done $v $w"
  done
done
