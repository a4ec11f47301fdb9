set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "not full_size" > gpurun_out/gpu_tests.log 2>&1; echo "PYTEST EXIT $?" >> gpurun_out/gpu_tests.log
tail -4 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
