set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for wh in "19 19" "18 19" "19 20" "19 21" "19 22" "18 21" "20 21"; do
  set -- $wh
  ZKP_WINDOW_BITS_W=$1 ZKP_WINDOW_BITS_H=$2 timeout -k 10 200 python bench.py --steps 6 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_c$1_$2.log 2>&1
done
