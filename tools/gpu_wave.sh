#!/bin/bash
# wave-lane bring-up: GPU parity tests on the default library, then A/B timings of
# the fast-lane variants (each checked against the oracle), then the bench line.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on() { case "$1" in 0|1) return 0 ;; *) echo "STOP: exit status $1"; exit "$1" ;; esac; }

if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
    rc=$?; echo "PYTEST EXIT $rc" >> gpurun_out/gpu_tests.log; tail -6 gpurun_out/gpu_tests.log
    stop_on $rc
fi
V=$PWD/tcpreplay_amd/lib/var
for v in ${VARIANTS:-default block w6b3 w4b3 w4b4}; do
    case $v in
        default) unset TCPEDIT_HIP_LIB TCPEDIT_HIP_FAST_KIND ;;
        block) unset TCPEDIT_HIP_LIB; export TCPEDIT_HIP_FAST_KIND=block ;;
        *) export TCPEDIT_HIP_LIB=$V/libtcpedit_hip_$v.so; unset TCPEDIT_HIP_FAST_KIND ;;
    esac
    AB_TAG=$v timeout -k 10 200 python -u tools/ab.py > gpurun_out/ab_$v.txt 2>&1
    rc=$?; grep -v "^$" gpurun_out/ab_$v.txt | tail -4; [ $rc -eq 0 ] || { echo "AB $v exit $rc"; exit $rc; }
done
unset TCPEDIT_HIP_LIB TCPEDIT_HIP_FAST_KIND
if [ -z "$SKIP_BENCH" ]; then
    timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
fi
echo DONE
