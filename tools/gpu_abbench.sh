#!/bin/bash
# bench.py at full size for library variants (diagnostic): AB_VARIANTS (names under
# tcpreplay_amd/lib/abvar -- copy them there from lib/var, which no GPU run receives;
# "base" = the in-tree library), AB_WLS workloads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F="--steps 20 --warmup 3 --extra= --no-cpu-baseline --no-e2e --no-device-index --no-packet-latency ${AB_NOVERIFY:+--no-verify}"
for v in ${AB_VARIANTS:-base}; do
  for w in ${AB_WLS:-c4}; do
    if [ "$v" = base ]; then L=tcpreplay_amd/lib/libtcpedit_hip.so; else L=tcpreplay_amd/lib/abvar/libtcpedit_hip_$v.so; fi
    TCPEDIT_HIP_LIB=$L timeout -k 10 300 python3 bench.py --workload $w $F > gpurun_out/abb_${v}_$w.json 2> gpurun_out/abb_${v}_$w.err || { tail -5 gpurun_out/abb_${v}_$w.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print(sys.argv[2], sys.argv[3], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'], 'pipe_ms', r['pipeline_ms'])" gpurun_out/abb_${v}_$w.json $v $w
    if [ -n "$AB_PMC" ]; then
      TCPEDIT_HIP_LIB=$L timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/abw_${v}_$w -o run -- python3 bench.py --workload $w $F > /dev/null 2>&1 || exit 1
      python3 -c "
import csv,statistics,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open(sys.argv[1])) if 'te_wave' in r['Kernel_Name'] and r['Counter_Name']=='WRITE_SIZE']
print(sys.argv[2], sys.argv[3], 'WRITE_SIZE bytes', statistics.median(v)*1024)" gpurun_out/abw_${v}_$w/run_counter_collection.csv $v $w
    fi
  done
done
