#!/bin/bash
# bench.py at full size with an environment knob on and off (diagnostic): AB_ENV (NAME),
# AB_VALS (values, "-" = unset), AB_WLS workloads; outputs oracle-checked unless AB_NOVERIFY
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--steps 200 --warmup 10 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency ${AB_NOVERIFY:+--no-verify}"
for v in ${AB_VALS:-- 1}; do
  for w in ${AB_WLS:-c2}; do
    if [ "$v" = - ]; then unset "$AB_ENV"; else export "$AB_ENV=$v"; fi
    timeout -k 10 300 python3 bench.py --workload $w $F > gpurun_out/abe_${v}_$w.json 2> gpurun_out/abe_${v}_$w.err || { tail -5 gpurun_out/abe_${v}_$w.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print(sys.argv[2], sys.argv[3], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'], 'ms_per_step', j['ms_per_step'])" gpurun_out/abe_${v}_$w.json $v $w
  done
done
