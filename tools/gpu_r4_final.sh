# round 4 evidence (one gpurun call): smoke(), the default bench line, then rocprofv3 kernel
# stats + FETCH/WRITE PMC passes for C2 (its bench run includes the window-mode launches), C4
# and the generic-lane mtu line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/r4_$name.log" 2>&1; local rc=$?
    tail -3 "gpurun_out/r4_$name.log"
    [ $rc = 0 ] || { echo "step $name ended with $rc: stopping"; exit $rc; }
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 700 python bench.py
cp gpurun_out/r4_bench.log gpurun_out/r4_bench.json
ROUND=r04 WLS="c2 c4 mtu" bash tools/gpu_prof.sh
