# round 3: verify-before-return GPU tests, isolated plan timings, and the proof with the witness
# plan on the high-priority stream (ZKP_WPLAN_HI=1) vs the low-priority s2 vs the rocprim plan
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gt_verify.log 2>&1
timeout -k 10 300 python tools/probe/wplan_bench.py 10 > gpurun_out/wplan_bench.json 2> gpurun_out/wplan_bench.err
rm -f gpurun_out/wplan_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
row() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g1_abc"], s["ntt_quotient"], d["roofline"]["avg_launch_ms"])'; }
for i in 1 2; do
  for cfg in "ZKP_NONE=1" "ZKP_WPLAN_HI=1" "ZKP_W_SORT=rocprim" "ZKP_W_SORT=rocprim ZKP_WPLAN_HI=1"; do
    env $cfg timeout -k 10 300 $B > gpurun_out/b_wp.log 2>&1
    echo "$cfg $(tail -1 gpurun_out/b_wp.log | row)" >> gpurun_out/wplan_ab.txt
  done
done
