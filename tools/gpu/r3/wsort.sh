# round 3: the hand-written witness-plan sort -- GPU suite (incl. the configs[3]/[4]-shape
# parity tests), then an A/B of the witness plan (ZKP_W_SORT=rocprim = the round-2 onesweep plan)
# and a kernel trace of the default proof (no rocprim / hipcub kernels expected)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gt_r3.log 2>&1
rm -f gpurun_out/wsort_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  ZKP_W_SORT=rocprim timeout -k 10 300 $B > gpurun_out/b_ws.log 2>&1
  echo "rocprim $(tail -1 gpurun_out/b_ws.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"]["msm_g1_abc"], d["roofline"]["avg_launch_ms"], d["roofline"]["algorithmic_work_per_launch"]["mixed_adds"])')" >> gpurun_out/wsort_ab.txt
  timeout -k 10 300 $B > gpurun_out/b_ws.log 2>&1
  echo "hsort   $(tail -1 gpurun_out/b_ws.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"]["msm_g1_abc"], d["roofline"]["avg_launch_ms"], d["roofline"]["algorithmic_work_per_launch"]["mixed_adds"])')" >> gpurun_out/wsort_ab.txt
done
W=/tmp/zkp_prof
rm -rf $W && mkdir -p $W
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0 > gpurun_out/prof/conc.log 2>&1
cp $W/conc/run_kernel_stats.csv gpurun_out/prof/conc_kernel_stats_r3.csv
(cd tools/prof && python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/prof/timeline_r3.txt)
rm -rf $W
