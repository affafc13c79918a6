# A/B/... on one box with the in-tree library: the default timing loop under different ZKP_MSM settings
# (arm "none" = unset), alternating, N rounds; tools/gpu/ab_summary.py tabulates
#   bash tools/gpu/abenv.sh <tag> <rounds> <arm> [arm ...]     e.g.  abenv.sh qg 3 none qgate=1 qgate=2
source "$(dirname "$0")/common.sh"
N=${1:?rounds}; shift
for i in $(seq 1 $N); do
  for arm in "$@"; do
    if [ "$arm" = none ]; then unset ZKP_MSM; else export ZKP_MSM=$arm; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0 > "$O/ab_${arm}_$i.json" 2> "$O/ab_${arm}_$i.err"
  done
done
unset ZKP_MSM
echo abenv done
