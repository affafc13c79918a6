# round 3: NTT stage-root tables (ZKP_NTT_RTAB) -- NTT parity tests, isolated A/B, whole-proof A/B,
# then the kernel traces (concurrent + serial) of the default proof for profiles/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 120 --timeout-method thread -k "ntt or quotient or golden or bit_exact" > gpurun_out/gt_ntt.log 2>&1
timeout -k 10 400 python tools/probe/ntt_env_ab.py 3 "ZKP_NTT_RTAB=0" "ZKP_NTT_RTAB=1" > gpurun_out/ntt_rtab_ab.txt 2>&1
rm -f gpurun_out/rtab_proof_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for cfg in "ZKP_NTT_RTAB=0" "ZKP_NTT_RTAB=1"; do
    env $cfg timeout -k 10 300 $B > gpurun_out/b_rt.log 2>&1
    echo "$cfg $(tail -1 gpurun_out/b_rt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"]["ntt_quotient"])')" >> gpurun_out/rtab_proof_ab.txt
  done
done
W=/tmp/zkp_prof
rm -rf $W && mkdir -p $W
BP="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/conc -o run -- $BP > gpurun_out/prof/conc.log 2>&1
ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/ser -o run -- $BP > gpurun_out/prof/ser.log 2>&1
cp $W/conc/run_kernel_stats.csv gpurun_out/prof/conc_kernel_stats_r3b.csv
cp $W/ser/run_kernel_stats.csv gpurun_out/prof/ser_kernel_stats_r3b.csv
cp gpurun_out/prof/conc.log gpurun_out/prof/bench_line_rocprof_r3b.log
(cd tools/prof && python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/prof/timeline_r3b.txt && python3 breakdown.py $W/ser/run_kernel_stats.csv > ../../gpurun_out/prof/serial_breakdown_r3b.txt)
rm -rf $W
