# round 3: the all-uniform-witness line (witness MSMs with ~96 M digits each, G2 on the critical
# path) for HEAD (cur), HEAD without the G2 chained pairs (nog2) and the pre-chain library (base)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/bool0_ab.txt
B="python bench.py --bool-pct 0 --steps 8 --warmup 2 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for lib in cur nog2 base; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_b0.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_b0.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g1_abc"], s["msm_g2"], s["msm_g1_h"], d["all_proofs_ok"])')" >> gpurun_out/bool0_ab.txt
  done
done
