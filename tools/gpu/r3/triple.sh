# round 3: ZKP_MUL_PAIRS=2 (PPP/Q/ZZ3 triple, ZZZ3 beside the Y3 sum of products) vs pairs (cur)
# round 3: independent product pairs of the mixed addition in lockstep (mul_pair / sqr_pair) vs HEAD:
# parity (kernels + golden proofs + full-size proof), whole-proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_tri.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k "venmo_full_proof" > gpurun_out/gt_tri_full.log 2>&1
rm -f gpurun_out/tri_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0"
for i in 1 2; do
  for lib in cur tri; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_p.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; k=d["kernels_config1"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["isolated_launch"]["avg_launch_ms"], k["msm_g1_2^20_ms"], d["all_proofs_ok"])')" >> gpurun_out/tri_ab.txt
  done
done
timeout -k 10 120 ./tools/ubench/mul_chain > gpurun_out/mul_chain3.txt 2>&1
