# round 5: the all-uniform witness (it takes the second witness configuration, whose buckets fill evenly
# like the H plan's): witness-plan tasks of 48 vs 32, alternated 3 rounds (staged bench, --bool-pct 0)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
for i in 1 2 3; do
  for arm in base tw48; do
    if [ $arm = base ]; then E="ZKP_X=1"; else E="ZKP_MSM=task_w=48"; fi
    env $E timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --bool-pct 0 > gpurun_out/r5/uni_${arm}_$i.json 2> gpurun_out/r5/uni_${arm}_$i.err
    echo "uni $arm $i $(tail -1 gpurun_out/r5/uni_${arm}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["all_proofs_ok"])')"
  done
done
