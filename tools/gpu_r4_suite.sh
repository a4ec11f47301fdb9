# round 4: the whole GPU suite (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4_suite.log 2>&1; rc=$?
tail -4 gpurun_out/r4_suite.log
exit $rc
