# round 3: product-column chains via empty-asm barriers (the compiler keeps real mads and interleaves
# chains) vs inline-asm mads; G1 accumulation only (B2) or every field (B2ALL).  Microbenchmark,
# parity of both variant libraries, isolated NTT A/B, whole-proof A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/mul_chain > gpurun_out/mul_chain2.txt 2>&1
for v in B2 B2ALL; do
  ZKP_LIB_PATH=$PWD/ablib/lib_$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_$v.log 2>&1
done
timeout -k 10 300 python tools/probe/ntt_ab.py 2 ablib/lib_asm.so ablib/lib_B2ALL.so > gpurun_out/bar_ntt_ab.txt 2>&1
rm -f gpurun_out/bar_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0"
for i in 1 2; do
  for lib in asm B2 B2ALL; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_bar.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_bar.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; k=d["kernels_config1"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["isolated_launch"]["avg_launch_ms"], k["msm_g1_2^20_ms"], k["ntt_roofline"]["2^23 (Venmo domain)"]["ms"], s["msm_g2"], d["all_proofs_ok"])')" >> gpurun_out/bar_ab.txt
  done
done
