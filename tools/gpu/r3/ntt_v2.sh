# round 3: NTT v2 variants -- Shoup twiddles / coset key (TWSHOUP), stage roots from a global table
# (GROOTS), 4 waves per SIMD (WPE=4).  Parity tests of the in-tree library, then the isolated A/B of
# the variant libraries in ablib/ (A = HEAD before the change).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 120 --timeout-method thread -k "ntt or quotient or golden or bit_exact" > gpurun_out/gt_ntt2.log 2>&1
timeout -k 10 600 python tools/probe/ntt_ab.py 2 ablib/lib_ntt_A.so ablib/lib_ntt_B.so ablib/lib_ntt_C.so ablib/lib_ntt_D.so ablib/lib_ntt_E.so > gpurun_out/ntt_v2_ab.txt 2>&1
