set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/prep_tests.log 2>&1; rc=$?; tail -30 gpurun_out/prep_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/prep_probe.py > gpurun_out/prep_probe.txt 2>&1 || { tail gpurun_out/prep_probe.txt; exit 1; }
cat gpurun_out/prep_probe.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_prep -- python $GRAFT_REPO_ROOT/tools/prep_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_prep.log 2>&1 || echo PROF FAILED
find $GRAFT_REPO_ROOT/gpurun_out/prof_prep -name "*stats*"
