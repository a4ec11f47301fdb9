# e2e A/B: the in-tree library (6 pipeline slots) against lib/abvar's 3-slot build, fresh
# processes in turn (tools/e2e_ctx_probe.py plain: C2 pinned, median of 9), plus the
# pipelined tests under the new default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pipelined or pipeline or chunk" \
    tests/test_q8.py tests/test_device_index.py > gpurun_out/slots_tests.log 2>&1
rc=$?; tail -2 gpurun_out/slots_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4; do
  for v in base slots3; do
    if [ $v = base ]; then L=tcpreplay_amd/lib/libtcpedit_hip.so; else L=tcpreplay_amd/lib/abvar/libtcpedit_hip_$v.so; fi
    echo -n "$v: "; TCPEDIT_HIP_LIB=$L timeout -k 10 100 python tools/e2e_ctx_probe.py plain 2>/dev/null || exit 1
  done
done
