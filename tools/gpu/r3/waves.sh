# round 3: G1 accumulation at 5 / 6 waves per SIMD (ZKP_G1_ACC_WAVES, spills) and Fr product chains
# in the NTT (ZKP_CHAIN_FR) vs HEAD (cur): isolated NTT A/B, whole-proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZKP_LIB_PATH=$PWD/ablib/lib_frch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ntt or quotient" > gpurun_out/gt_frch.log 2>&1
timeout -k 10 300 python tools/probe/ntt_ab.py 3 ablib/lib_cur.so ablib/lib_frch.so > gpurun_out/frch_ntt_ab.txt 2>&1
rm -f gpurun_out/waves_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0"
for i in 1 2; do
  for lib in cur w5 w6 frch; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_w.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; k=d["kernels_config1"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["isolated_launch"]["avg_launch_ms"], k["msm_g1_2^20_ms"], k["ntt_roofline"]["2^23 (Venmo domain)"]["ms"], d["all_proofs_ok"])')" >> gpurun_out/waves_ab.txt
  done
done
