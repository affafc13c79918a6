# H-plan task size sweep (whole-bucket tasks shorten the H finish's merge chains), alternating with the default.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/tasks2_summary.txt
for cfg in "ZKP_TASK_H=32" "ZKP_TASK_H=256" "ZKP_TASK_H=512" "ZKP_TASK_H=32" "ZKP_TASK_H=256" "ZKP_TASK_H=160"; do
  env $cfg timeout -k 10 300 python bench.py --steps 12 --warmup 2 --cpu-baseline none --no-kernels --batch 0 > gpurun_out/b_t.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/b_t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"])')" >> gpurun_out/tasks2_summary.txt
done
