#!/bin/bash
# bench.py's end_to_end line (measured in a child process) against a standalone probe, then the default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
show() { python3 -c "import json,sys; e=json.load(open(sys.argv[1]))['end_to_end']; print(sys.argv[2], 'pinned', e['ms'], 'pageable', e['pageable']['ms'], 'floor', e['copy_floor_ms'])" "$1" "$2"; }
B="--extra= --no-cpu-baseline --no-device-index --no-packet-latency"
timeout -k 10 300 python3 bench.py $B --steps 5 --warmup 1 > gpurun_out/e2eb_1.json 2> gpurun_out/e2eb_1.err && show gpurun_out/e2eb_1.json "steps 5" || exit 1
timeout -k 10 300 python3 tools/e2e_host_ab.py 2 torch || exit 1
timeout -k 10 500 python3 bench.py > gpurun_out/e2eb_3.json 2> gpurun_out/e2eb_3.err && show gpurun_out/e2eb_3.json "full" || exit 1
