# widened wave lane: GPU suite, then the new bench extras and a C3 instance A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -8 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --extra c3,seed,hdr,vdel,efcs,c5 --no-cpu-baseline --no-e2e > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err || { tail -20 gpurun_out/bench_wide.err; exit 1; }
cat gpurun_out/bench_wide.json
TCPEDIT_HIP_WAVE_FEAT=15 timeout -k 10 300 python bench.py --workload c3 --steps 50 --extra '' --no-cpu-baseline --no-e2e > gpurun_out/bench_c3_f15.json 2>&1 || exit 1
cat gpurun_out/bench_c3_f15.json
