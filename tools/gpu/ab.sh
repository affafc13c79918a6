# A/B on one box: the default timing loop with a base library (ZKP_LIB_PATH, built on the CPU into the
# git-ignored tools/gpu/libs/: ./abtest is gpurun-ignored and never reaches the box) against the in-tree
# library, alternating, N rounds; tools/gpu/ab_summary.py tabulates
#   bash tools/gpu/ab.sh <tag> [rounds=2] [base .so=tools/gpu/libs/base.so] [extra bench args]
source "$(dirname "$0")/common.sh"
N=${1:-2}; shift || true
BASE=${1:-$PWD/tools/gpu/libs/base.so}; shift || true
for i in $(seq 1 $N); do
  ZKP_LIB_PATH=$BASE timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0 "$@" > $O/ab_base_$i.json 2> $O/ab_base_$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0 "$@" > $O/ab_new_$i.json 2> $O/ab_new_$i.err
done
echo ab done
