# round 3 evidence (one gpurun call): GPU suite, smoke(), the default bench line, then
# rocprofv3 kernel stats + FETCH/WRITE PMC passes for C2, C4 and the generic-lane mtu line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { # name seconds cmd...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/r3_$name.log" 2>&1; local rc=$?
    tail -3 "gpurun_out/r3_$name.log"
    [ $rc = 0 ] || { echo "step $name ended with $rc: stopping"; exit $rc; }
}
step suite 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cp gpurun_out/r3_bench.log gpurun_out/r3_bench.json
ROUND=r03 WLS="c2 c4 mtu" bash tools/gpu_prof.sh
