# the file-based / segment sharded path on the GPU, and the C4 job at its real size
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_dist.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/dist_gpu.log 2>&1; rc=$?; tail -12 gpurun_out/dist_gpu.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u bench.py --workload c4 --strong --steps 20 --warmup 2 > gpurun_out/strong_c4.json 2> gpurun_out/strong_c4.err || { echo STRONG FAILED; tail -20 gpurun_out/strong_c4.err; exit 1; }
cat gpurun_out/strong_c4.json
