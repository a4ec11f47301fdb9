# A/B of the balanced small-batch tile cut (TCPEDIT_HIP_BALANCE=0: the greedy cut), then the fast-lane parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 3000 --warmup 20 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency"
for i in 1 2 3; do
  for bal in 0 1; do
    TCPEDIT_HIP_BALANCE=$bal timeout -k 10 120 $B > gpurun_out/bal_${bal}_$i.json 2>gpurun_out/bal.err || { tail gpurun_out/bal.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bal_${bal}_$i.json'));r=d['roofline'];print('bal=$bal', r['kernel_ms'], r['frac'], d['ms_per_step'])"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_fast_lane.py tests/test_gpu_parity.py tests/test_shrink.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bal_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bal_tests.log; exit $rc
