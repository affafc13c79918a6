# round 3: the H MSM in two point-range halves (ZKP_H_HALVES=2: second half's plan beside the first
# half's accumulation, first half's finish beside the second's).  Parity of the in-tree library
# (kernels, golden proofs incl. knob variants, full-size proofs vs oracle/cpu, configs tests), then
# whole-proof A/B: base (HEAD), G1 asm chains only, G1 asm + halves, G1 asm + halves off.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_hh.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k "venmo_full_proof" > gpurun_out/gt_hh_full.log 2>&1
rm -f gpurun_out/hh_ab.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for cfg in "base:" "asm:" "new:" "new:ZKP_H_HALVES=1"; do
    lib=${cfg%%:*}; e=${cfg#*:}
    env $e ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_hh.log 2>&1
    echo "$lib $e $(tail -1 gpurun_out/b_hh.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], s["ntt_quotient"], s["msm_g1_h"], s["msm_g2"], d["all_proofs_ok"])')" >> gpurun_out/hh_ab.txt
  done
done
