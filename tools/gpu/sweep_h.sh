# H-plan window bits: 20 (19-bit keys, 3 sort passes, 13 windows) vs 19 (2 passes, 14 windows)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for h in 19 20 19 20; do
  ZKP_WINDOW_BITS_H=$h timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bh_$h.log 2>&1
done
