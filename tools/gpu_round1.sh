#!/bin/bash
# One gpurun call: GPU parity tests, bench, rocprofv3 kernel-trace stats and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic figure.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
WL=${WL:-c2}

step_ok() {  # $1 = exit status; 0/1 (test failures) may continue, anything else stops
    case "$1" in 0|1) return 0 ;; *) echo "STOP: exit status $1"; exit "$1" ;; esac
}

if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 700 python -m pytest tests -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
    rc=$?; echo "PYTEST EXIT $rc" >> gpurun_out/gpu_tests.log
    tail -5 gpurun_out/gpu_tests.log
    step_ok $rc
fi

timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }

[ -n "$SKIP_PROF" ] && exit 0
P="python3 bench.py --workload $WL --steps 20 --warmup 2 --extra= --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${R}_${WL} -o run -- $P \
    > gpurun_out/prof_${R}_${WL}.log 2>&1 || { echo "kernel-trace FAILED"; tail -20 gpurun_out/prof_${R}_${WL}.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${R}_${WL} -o run -- $P \
    > gpurun_out/pmc_fetch_${R}_${WL}.log 2>&1 || { echo "pmc FETCH FAILED"; tail -20 gpurun_out/pmc_fetch_${R}_${WL}.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${R}_${WL} -o run -- $P \
    > gpurun_out/pmc_write_${R}_${WL}.log 2>&1 || { echo "pmc WRITE FAILED"; tail -20 gpurun_out/pmc_write_${R}_${WL}.log; exit 1; }
find gpurun_out/prof_${R}_${WL} gpurun_out/pmc_*_${R}_${WL} -name "*.csv"
echo DONE
