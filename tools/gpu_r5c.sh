# tcpprep auto+filter GPU parity, then C3/C4 wave-lane phase stamps (TE_WK_STAMPS variant in lib/abvar)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_tcpprep_gpu.py \
    > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
TCPEDIT_HIP_LIB=tcpreplay_amd/lib/abvar/libtcpedit_hip_stamps.so timeout -k 10 240 python -u tools/c4_stamps.py \
    > gpurun_out/r5c_stamps.log 2>&1
rc=$?; grep -c wstamps gpurun_out/r5c_stamps.log; grep "==" gpurun_out/r5c_stamps.log; exit $rc
