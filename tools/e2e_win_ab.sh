# window-mode pipeline: how far the host enqueues ahead (diagnostics)
set -o pipefail
mkdir -p gpurun_out
for v in "TCPEDIT_HIP_PIPE_WIN_AHEAD=2" "TCPEDIT_HIP_PIPE_NO_WIN=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/e2e_probe.py ${1:-2,4,8} 1 > gpurun_out/e2e_win_ab.txt 2>&1 || { tail -5 gpurun_out/e2e_win_ab.txt; exit 1; }
  grep -v "^pipe" gpurun_out/e2e_win_ab.txt | grep pinned
done
