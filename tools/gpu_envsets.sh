#!/bin/bash
# bench.py at full size under sets of environment knobs (diagnostic): AB_SETS (space-separated
# sets, each NAME=VAL[,NAME=VAL...] or "none"), AB_WLS workloads; outputs oracle-checked
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--steps 200 --warmup 10 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency ${AB_NOVERIFY:+--no-verify}"
for set in ${AB_SETS:-none}; do
  for w in ${AB_WLS:-c5}; do
    ENVS=()
    [ "$set" = none ] || IFS=, read -ra ENVS <<< "$set"
    tag=$(echo "$set" | tr ',=' '__')
    env "${ENVS[@]}" timeout -k 10 300 python3 bench.py --workload $w $F > gpurun_out/abs_${tag}_$w.json 2> gpurun_out/abs_${tag}_$w.err || { tail -5 gpurun_out/abs_${tag}_$w.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print(sys.argv[2], sys.argv[3], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'])" gpurun_out/abs_${tag}_$w.json "$set" $w
  done
done
