# Scheduling sweep with the look-back-free H plan: CU-reserved witness streams, G2 gating.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/reserve_summary.txt
for cfg in "ZKP_RESERVE_CUS=0" "ZKP_RESERVE_CUS=32" "ZKP_RESERVE_CUS=64" "ZKP_RESERVE_CUS=32 ZKP_SCHED=4" "ZKP_RESERVE_CUS=16" "ZKP_RESERVE_CUS=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_res.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/b_res.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"])')" >> gpurun_out/reserve_summary.txt
done
