# round 3: G2 (Fq2) products as lockstep pairs of chained sums of products (ZKP_CHAIN_G2, g2c) vs
# HEAD (cur): parity (kernel + prove tests), whole-proof A/B with the config-1 kernels
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZKP_LIB_PATH=$PWD/ablib/lib_g2c.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_g2c.log 2>&1
rm -f gpurun_out/g2c_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for lib in cur g2c; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_g2.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_g2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g2"], d["all_proofs_ok"])')" >> gpurun_out/g2c_ab.txt
  done
done
