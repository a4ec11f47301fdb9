set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; echo "PYTEST EXIT $?" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_c2 -- python bench.py --steps 50 --warmup 2 --extra '' --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || echo PROF FAILED
find gpurun_out/prof_c2 -name "*stats*" | head
