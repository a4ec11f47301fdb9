#!/bin/bash
# window mode (fused line) with TCPEDIT_HIP_WIN_BALANCE off / on, alternating (diagnostic)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--steps 200 --warmup 10 --extra= --no-cpu-baseline --no-e2e --no-packet-latency --no-verify"
for i in 1 2 3; do
  for v in 0 1; do
    for w in ${WLS:-c2 c2x10}; do
      TCPEDIT_HIP_WIN_BALANCE=$v timeout -k 10 300 python3 bench.py --workload $w $F > gpurun_out/wb_${v}_$w.json 2> gpurun_out/wb_${v}_$w.err || { tail -5 gpurun_out/wb_${v}_$w.err; exit 1; }
      python3 -c "import json,sys; j=json.load(open(sys.argv[1])); f=j.get('fused',{}); print(sys.argv[2], sys.argv[3], 'fused', f.get('frac_hbm_peak'), 'same', f.get('same_bytes_as_exact_path'))" gpurun_out/wb_${v}_$w.json $v $w
    done
  done
done
