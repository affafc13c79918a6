# round 3: re-sweep of the MSM task / reduction knobs at HEAD (the chained / paired arithmetic
# changed the cost balance between accumulation, merges and the bucket reduction)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/knobs3.txt
B="python bench.py --steps 16 --warmup 2 --cpu-baseline none --batch 0 --no-kernels"
run() {
  env "$@" timeout -k 10 300 $B > gpurun_out/b_k.log 2>&1
  echo "$* $(tail -1 gpurun_out/b_k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g1_abc"], s["msm_g2"], s["msm_g1_h"], d["all_proofs_ok"])')" >> gpurun_out/knobs3.txt
}
for i in 1 2 3; do
  run ZKP_NONE=0
  run ZKP_TASK_H=48
  run ZKP_TASK_H=48 ZKP_TASK_W=48
done
