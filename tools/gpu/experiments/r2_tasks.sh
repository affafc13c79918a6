# Task-size sweep with length-ordered tasks.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/tasks_summary.txt
for cfg in "ZKP_TASK_H=32" "ZKP_TASK_H=64" "ZKP_TASK_H=128" "ZKP_TASK_W=64" "ZKP_TASK_W=64 ZKP_TASK_H=64" "ZKP_TASK_W=24" "ZKP_TASK_H=32"; do
  env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_t.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/b_t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"])')" >> gpurun_out/tasks_summary.txt
done
