# round 3: field product columns as inline-asm dependent mad chains (ZKP_ASM_MAC) -- kernel/prove
# parity of the in-tree library, isolated NTT + MSM A/B and whole-proof A/B vs the base library
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_asm.log 2>&1
ZKP_LIB_PATH=$PWD/ablib/lib_asm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k "venmo_full_proof" > gpurun_out/gt_asm_full.log 2>&1
rm -f gpurun_out/asm_proof_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0"
for i in 1 2; do
  for lib in ablib/lib_base.so ablib/lib_asm.so; do
    ZKP_LIB_PATH=$PWD/$lib timeout -k 10 300 $B > gpurun_out/b_asm.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_asm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_config1"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["isolated_launch"]["avg_launch_ms"], k["msm_g1_2^20_ms"], k["ntt_roofline"]["2^23 (Venmo domain)"]["ms"])')" >> gpurun_out/asm_proof_ab.txt
  done
done
