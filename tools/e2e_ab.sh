# e2e A/B over the pipeline's modes and chunk sizes (diagnostics): the window mode (default
# for size-preserving wave-lane configs), the device record index, early D2H off
set -o pipefail
mkdir -p gpurun_out
for v in "" "TCPEDIT_HIP_PIPE_NO_WIN=1" "TCPEDIT_HIP_PIPE_NO_WIN=1 TCPEDIT_HIP_PIPE_NO_EARLY=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/e2e_probe.py ${1:-2,4,8,16} 1 > gpurun_out/e2e_ab.txt 2>&1 || { tail -5 gpurun_out/e2e_ab.txt; exit 1; }
  grep -v "^pipe" gpurun_out/e2e_ab.txt | grep pinned
  grep "^pipe" gpurun_out/e2e_ab.txt | sort | uniq -c | sort -rn | head -3
done
