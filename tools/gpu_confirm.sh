set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "PYTEST EXIT $?" >> gpurun_out/gpu_tests.log
tail -4 gpurun_out/gpu_tests.log
grep -q "PYTEST EXIT 0" gpurun_out/gpu_tests.log || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
