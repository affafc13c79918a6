# round 3: stream gates re-measured with the chained G1 accumulation (contended launches got
# cheaper, the lone H accumulation did not): G2 MSM gated on the quotient (ZKP_SCHED=4) or on the
# H plan too (=5), witness accumulations gated on the quotient (=1), G2 finish on the finish stream
# after the H plan (ZKP_G2_FINISH_GATE=2)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/sched_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for cfg in "ZKP_NONE=0" "ZKP_SCHED=4" "ZKP_SCHED=5" "ZKP_SCHED=1" "ZKP_G2_FINISH_GATE=2"; do
    env $cfg timeout -k 10 300 $B > gpurun_out/b_s.log 2>&1
    echo "$cfg $(tail -1 gpurun_out/b_s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], s["ntt_quotient"], s["msm_g1_h"], s["msm_g2"], d["all_proofs_ok"])')" >> gpurun_out/sched_ab.txt
  done
done
