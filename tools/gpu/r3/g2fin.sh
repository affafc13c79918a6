# round 3: the G2 finish on the high-priority finish stream without a gate (ZKP_G2_FINISH_GATE=3) vs
# on s1 (default): with the chained kernels its subset-sum launch starved behind the H accumulation
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZKP_G2_FINISH_GATE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread -k "bit_exact" > gpurun_out/gt_g2f.log 2>&1
rm -f gpurun_out/g2f_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2 3; do
  for cfg in "ZKP_G2_FINISH_GATE=0" "ZKP_G2_FINISH_GATE=3"; do
    env $cfg timeout -k 10 300 $B > gpurun_out/b_g2f.log 2>&1
    echo "$cfg $(tail -1 gpurun_out/b_g2f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g2"], s["msm_g1_h"], d["all_proofs_ok"])')" >> gpurun_out/g2f_ab.txt
  done
done
