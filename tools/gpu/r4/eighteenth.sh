# round 4, eighteenth call: as seventeenth.sh, with the batch line warmed up by two proofs per worker
# (instead of two in all)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/r4/bfullw_$i.json 2> gpurun_out/r4/bfullw_$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/bshortw_$i.json 2> gpurun_out/r4/bshortw_$i.err
done
