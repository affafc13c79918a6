# round 3: one-limb screens of the mixed addition's exceptional-case tests (scr) vs HEAD (cur)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZKP_LIB_PATH=$PWD/ablib/lib_scr.so timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_scr.log 2>&1
rm -f gpurun_out/scr_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0"
for i in 1 2; do
  for lib in cur scr; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_scr.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_scr.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["msm_g2"], s["msm_g1_h"], d["kernels_config1"]["msm_g1_2^20_ms"], d["all_proofs_ok"])')" >> gpurun_out/scr_ab.txt
  done
done
