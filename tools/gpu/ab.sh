# A/B on one box: bench with abtest/libzkp_amd_base.so (ZKP_LIB_PATH) vs the in-tree library,
# alternating, N rounds (default 2).  Usage: bash tools/gpu/ab.sh [rounds] [extra bench args]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=${1:-2}; shift || true
for i in $(seq 1 $N); do
  ZKP_LIB_PATH=$PWD/abtest/libzkp_amd_base.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 "$@" > gpurun_out/ab_base_$i.log 2>&1
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 "$@" > gpurun_out/ab_new_$i.log 2>&1
done
