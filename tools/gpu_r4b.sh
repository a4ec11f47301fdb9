# round 4: window-pipeline A/B, window-mode stamps, a short bench (fused line)
set -o pipefail
mkdir -p gpurun_out
bash tools/e2e_win_ab.sh 1,2,4,8 > gpurun_out/e2e_win_ab_r4.txt 2>&1 || { echo E2E FAILED; tail -5 gpurun_out/e2e_win_ab_r4.txt; exit 1; }
cat gpurun_out/e2e_win_ab_r4.txt
TCPEDIT_HIP_LIB=$PWD/tcpreplay_amd/lib/var/libtcpedit_hip_stamps.so timeout -k 10 200 python tools/win_stamps.py > gpurun_out/win_stamps.txt 2>&1 || { echo STAMPS FAILED; tail -5 gpurun_out/win_stamps.txt; exit 1; }
grep -c wstamps gpurun_out/win_stamps.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --extra "" --no-cpu-baseline --no-e2e --no-packet-latency > gpurun_out/bench_r4b.json 2> gpurun_out/bench_r4b.err || { echo BENCH FAILED; tail -5 gpurun_out/bench_r4b.err; exit 1; }
cat gpurun_out/bench_r4b.json
