# A/B/... on one box with the in-tree library: the default timing loop under different environments,
# alternating, N rounds; tools/gpu/ab_summary.py tabulates.  An arm is "none" (nothing set), "ZKP_<VAR>=<v>"
# (that variable) or anything else (ZKP_MSM=<arm>)
#   bash tools/gpu/abenv.sh <tag> <rounds> <arm> [arm ...]     e.g.  abenv.sh t 3 none w2=22 ZKP_INFLIGHT=2
source "$(dirname "$0")/common.sh"
N=${1:?rounds}; shift
for i in $(seq 1 $N); do
  for arm in "$@"; do
    case "$arm" in none) E=();; ZKP_*=*) E=("$arm");; *) E=("ZKP_MSM=$arm");; esac
    env "${E[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0 > "$O/ab_${arm}_$i.json" 2> "$O/ab_${arm}_$i.err"
  done
done
echo abenv done
