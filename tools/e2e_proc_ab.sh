# e2e per process (diagnostic): fresh processes in turn, default copies vs HSA_ENABLE_SDMA=0
# (blit kernels); prints each process's C2 pinned median
for i in 1 2 3 4; do
  for v in "X=1" "HSA_ENABLE_SDMA=0"; do
    echo -n "$v: "; env $v timeout -k 10 100 python tools/e2e_ctx_probe.py plain 2>/dev/null
  done
done
