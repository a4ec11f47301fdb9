# round 3 iteration (one gpurun call): device index + pipeline, tcpreplay-edit, parity subset, bench side lines.
# A step that times out, aborts or faults ends the call (no further GPU step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
fail=0
step() { # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/it_$name.log" 2>&1; local rc=$?
    tail -4 "gpurun_out/it_$name.log"
    case $rc in 0) ;; 1) fail=1 ;; *) echo "step $name ended with $rc: stopping"; exit $rc ;; esac
}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
TCPEDIT_HIP_IDX_DEBUG=1 TCPEDIT_HIP_PIPE_TRACE=1 step idx 300 $PYT tests/test_device_index.py
step replay 300 $PYT -m gpu tests/test_replay_edit.py
step par 700 $PYT -m gpu tests/test_abi.py tests/test_dlt_decoders.py tests/test_fast_lane.py tests/test_gpu_parity.py tests/test_q8.py tests/test_quirks.py tests/test_shrink.py
[ $fail = 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 200 --extra macseed,mtu,fz,c2x10 --no-cpu-baseline --no-packet-latency > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err || { tail -20 gpurun_out/it_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/it_bench.json'))
print('c2', d['roofline']['frac'], 'index', d['device_index'], 'e2e', d.get('end_to_end'))
for k,v in d['extra_configs'].items(): print(k, v.get('frac_hbm_peak'), v.get('kernel_frac_hbm_peak'), v.get('verified'))"
