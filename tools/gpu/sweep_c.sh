set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 18 19 21 22; do
  ZKP_WINDOW_BITS=$c timeout -k 10 200 python bench.py --steps 6 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_c$c.log 2>&1
done
