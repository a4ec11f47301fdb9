# device record index: its tests, then the bench's device_index line (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TCPEDIT_HIP_IDX_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_device_index.py -x -v --timeout 120 --timeout-method thread > gpurun_out/idx_tests.log 2>&1; rc=$?; tail -15 gpurun_out/idx_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --extra c2x10 --no-cpu-baseline --no-e2e --no-packet-latency > gpurun_out/idx_bench.json 2> gpurun_out/idx_bench.err || { tail -20 gpurun_out/idx_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/idx_bench.json')); print(d['roofline']['frac'], d['device_index'])"
