# A/B on one box: bench.py with library $1 (ZKP_LIB_PATH) vs the in-tree library, alternating,
# $2 rounds; extra bench args after.  Logs: gpurun_out/r4/ab_<tag>_{base,new}_<i>.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
LIB=$1; N=$2; TAG=$3; shift 3
for i in $(seq 1 $N); do
  ZKP_LIB_PATH=$PWD/$LIB timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line "$@" > gpurun_out/r4/ab_${TAG}_base_$i.json 2> gpurun_out/r4/ab_${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line "$@" > gpurun_out/r4/ab_${TAG}_new_$i.json 2> gpurun_out/r4/ab_${TAG}_new_$i.err
done
