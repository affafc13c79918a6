# Scheduling A/B with the look-back-free H plan: default vs G2 gated on the quotient (4) / H plan (5).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gt_sched.log 2>&1
for s in 0 4 5 0; do
  ZKP_SCHED=$s timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_sched$s.log 2>&1
  tail -1 gpurun_out/b_sched$s.log | cut -c1-200 >> gpurun_out/sched_summary.txt
done
ZKP_SCHED=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s4 -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/prof_s4.log 2>&1
