set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 0 5 3; do
  ZKP_ACC_WPE=$w timeout -k 10 200 python bench.py --steps 6 --warmup 2 --cpu-baseline none > gpurun_out/b_w$w.log 2>&1
done
