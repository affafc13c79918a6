# round 3: balanced H-plan windows -- kernel/prove tests with the knob, the full-size proof with it
# vs oracle/cpu, isolated H-plan timings and the whole-proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gt_hbal.log 2>&1
ZKP_H_BALANCED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -k "venmo_full_proof" > gpurun_out/gt_hbal_full.log 2>&1
rm -f gpurun_out/hbal_ab.txt
for i in 1 2 3; do
  for cfg in "ZKP_H_BALANCED=0" "ZKP_H_BALANCED=1"; do
    env $cfg timeout -k 10 300 python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels > gpurun_out/b_hb.log 2>&1
    echo "$cfg $(tail -1 gpurun_out/b_hb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"]["msm_g1_h"], d["config"]["msm"]["h"])')" >> gpurun_out/hbal_ab.txt
  done
done
