# round 3 iteration (one gpurun call): the named GPU tests (no -x), then the device index probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread "$@" > gpurun_out/iter.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|^E  " gpurun_out/iter.log | head -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/idx_probe.py 50 > gpurun_out/idx_probe.txt 2>&1 || { tail -20 gpurun_out/idx_probe.txt; exit 1; }
cat gpurun_out/idx_probe.txt
