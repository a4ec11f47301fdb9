#!/bin/bash
# SQ counters of the window-mode kernel against the exact path's (diagnostic): one --pmc pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/win_pmc -o run -- python3 tools/fused_probe.py 20 > gpurun_out/win_pmc.log 2>&1 || { tail -20 gpurun_out/win_pmc.log; exit 1; }
tail -4 gpurun_out/win_pmc.log
