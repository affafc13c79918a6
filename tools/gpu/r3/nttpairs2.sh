# round 3: NTT twiddle / coset-key products two elements at a time in lockstep (tp) vs HEAD (cur)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in tp; do
  ZKP_LIB_PATH=$PWD/ablib/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread -k "ntt or quotient or bit_exact" > gpurun_out/gt_$v.log 2>&1
done
timeout -k 10 400 python tools/probe/ntt_ab.py 3 ablib/lib_cur.so ablib/lib_tp.so > gpurun_out/nttt_ab.txt 2>&1
rm -f gpurun_out/nttt_proof.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for lib in cur tp; do
    ZKP_LIB_PATH=$PWD/ablib/lib_$lib.so timeout -k 10 300 $B > gpurun_out/b_np.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_np.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_last_proof"]; print(d["ms_per_step"], s["ntt_quotient"], d["all_proofs_ok"])')" >> gpurun_out/nttt_proof.txt
  done
done
