# round 5: the all-uniform witness with the second witness configuration at c = 20 (w + 2, default) vs
# c = 22 (w + 4), alternated 3 rounds (the staged bench on an all-uniform witness: auto-picks the second)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
for i in 1 2 3; do
  for w in 20 22; do
    ZKP_MSM=w2=$w timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --bool-pct 0 > gpurun_out/r5/w2_${w}_$i.json 2> gpurun_out/r5/w2_${w}_$i.err
    echo "w2=$w $i $(tail -1 gpurun_out/r5/w2_${w}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms_last_proof"].get("witness_config"))')"
  done
done
