# round 4, seventeenth call: the default bench twice and the short form twice on one box (is the batch
# line's lower ratio in full runs the box or the run?)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/r4/bfull_$i.json 2> gpurun_out/r4/bfull_$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/bshort_$i.json 2> gpurun_out/r4/bshort_$i.err
done
