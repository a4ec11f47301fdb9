# A/B: streaming (nontemporal) mode forced on/off vs the size rule
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in auto s0 s1 auto; do
  case $v in auto) env="";; s0) env="TCPEDIT_HIP_STREAM=0";; s1) env="TCPEDIT_HIP_STREAM=1";; esac
  env $env AB_TAG=$v timeout -k 10 200 python tools/ab.py c2 c2x10 c3 c5 c4 >> gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
done
cat gpurun_out/ab.log
