# round 3: NTT round-0 roots from the global table (R0G: 39 KiB LDS, 4 workgroups/CU at 128 VGPRs with
# spills) vs LDS roots.  Parity of both variant libraries, then the isolated A/B (F = HEAD).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in G H; do
  ZKP_LIB_PATH=$PWD/ablib/lib_ntt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ntt or quotient" > gpurun_out/gt_ntt_$v.log 2>&1
done
timeout -k 10 600 python tools/probe/ntt_ab.py 3 ablib/lib_ntt_F.so ablib/lib_ntt_G.so ablib/lib_ntt_H.so > gpurun_out/ntt_r0g_ab.txt 2>&1
