# round 3: NTT with the tile size known at compile time (LE = 10: one LDS address register per
# element, 142 -> 110 VGPRs) and the MODE-2 key buffer kept in registers.  Parity tests of the
# in-tree library, isolated A/B (A = HEAD, E = MODE-2 fix only, F = both), whole-proof A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 120 --timeout-method thread -k "ntt or quotient or golden or bit_exact" > gpurun_out/gt_ntt_le.log 2>&1
timeout -k 10 600 python tools/probe/ntt_ab.py 3 ablib/lib_ntt_A.so ablib/lib_ntt_E.so ablib/lib_ntt_F.so > gpurun_out/ntt_le_ab.txt 2>&1
rm -f gpurun_out/ntt_le_proof.txt
B="python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels"
for i in 1 2; do
  for lib in ablib/lib_ntt_A.so ablib/lib_ntt_F.so; do
    ZKP_LIB_PATH=$PWD/$lib timeout -k 10 300 $B > gpurun_out/b_le.log 2>&1
    echo "$lib $(tail -1 gpurun_out/b_le.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_last_proof"]["ntt_quotient"])')" >> gpurun_out/ntt_le_proof.txt
  done
done
