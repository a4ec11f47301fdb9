# end-to-end (host bytes -> host bytes) pipelined path: chunk ramp / walk stretch size A/B, stage trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 262144" "0 2097152" "1 2097152" "0 262144"; do
  set -- $cfg
  TCPEDIT_HIP_PIPE_RAMP=$1 TCPEDIT_HIP_WALK_PART=$2 timeout -k 10 300 python -u tools/e2e_probe.py > gpurun_out/e2e_$1_$2.log 2>&1 || { tail -20 gpurun_out/e2e_$1_$2.log; exit 1; }
  echo "ramp=$1 part=$2"; grep -E "^c2|^c3" gpurun_out/e2e_$1_$2.log | grep pinned
done
