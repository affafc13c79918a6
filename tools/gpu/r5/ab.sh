# round 5 A/B on one box, alternating arms N rounds: each arm is "tag:ENV=V[,ENV=V...]" (ZKP_LIB_PATH=
# relative to the repo for a library; "-" for none), run as the short staged bench.
# usage: bash tools/gpu/r5/ab.sh <rounds> <out-tag> <arm>... ; logs gpurun_out/r5/ab_<out-tag>_<arm>_<i>.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
N=$1; OUT=$2; shift 2
for i in $(seq 1 $N); do
  for arm in "$@"; do
    tag=${arm%%:*}; envs=${arm#*:}
    e=()
    if [ "$envs" != "-" ]; then IFS=',' read -ra kv <<< "$envs"; for x in "${kv[@]}"; do
      case $x in ZKP_LIB_PATH=*) e+=("ZKP_LIB_PATH=$PWD/${x#ZKP_LIB_PATH=}");; *) e+=("$x");; esac; done; fi
    env "${e[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r5/ab_${OUT}_${tag}_$i.json 2> gpurun_out/r5/ab_${OUT}_${tag}_$i.err
    echo "$OUT $tag $i $(tail -1 gpurun_out/r5/ab_${OUT}_${tag}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
  done
done
