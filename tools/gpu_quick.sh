# a short GPU check: the tests named on the command line (one pytest process, bounded)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread "$@" > gpurun_out/quick.log 2>&1
rc=$?
tail -30 gpurun_out/quick.log
exit $rc
