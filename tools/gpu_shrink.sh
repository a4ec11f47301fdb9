# size-reducing wave lane (VLAN pop, --efcs): its tests, the neighbours they touch, and
# the vdel / efcs bench lines (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_shrink.py tests/test_q8.py tests/test_gpu_parity.py tests/test_fast_lane.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/shrink_tests.log 2>&1; rc=$?; tail -15 gpurun_out/shrink_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 200 --extra vdel,efcs,c4 > gpurun_out/shrink_bench.json 2> gpurun_out/shrink_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/shrink_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/shrink_bench.json'))
for k,v in d['extra_configs'].items(): print(k, v.get('pipeline_ms'), v.get('kernel_ms'), v.get('frac_hbm_peak'), v.get('kernel_frac_hbm_peak'))
print('c2', d['roofline']['frac'])"
