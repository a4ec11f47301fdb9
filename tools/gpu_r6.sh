#!/bin/bash
# round-6 GPU check: the GPU suite, smoke, the default bench line, then SQ counters of the
# wave lane on WLS (default c4) -- one gpurun call
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_suite.sh > gpurun_out/suite_${TAG:-r6}.txt 2>&1 || { tail -30 gpurun_out/suite_${TAG:-r6}.txt; exit 1; }
tail -3 gpurun_out/gpu_tests.log
if [ -n "$WLS" ]; then
  rm -rf gpurun_out/pmc_sq_*
  SQ_VARIANTS=base WLS="$WLS" tools/gpu_sq.sh > gpurun_out/sq_${TAG:-r6}.txt 2>&1 && python3 tools/sq_summary.py > gpurun_out/sq_${TAG:-r6}_summary.txt
fi
