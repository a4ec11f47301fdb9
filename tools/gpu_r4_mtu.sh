# round 4: --mtu-trunc on the wave lane -- its parity tests, then the mtu bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mtu_wave.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/r4_mtu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r4_mtu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mtu --steps 50 --warmup 5 --extra= --no-cpu-baseline --no-e2e \
    --no-device-index --no-packet-latency > gpurun_out/r4_mtu_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4_mtu_bench.log | cut -c1-900
exit $rc
