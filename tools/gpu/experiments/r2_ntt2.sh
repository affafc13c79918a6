# NTT swizzle check: NTT/quotient/golden GPU tests on the in-tree library, variant timing, LDS counters
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ntt or quotient or golden" > gpurun_out/ntt_tests.log 2>&1
timeout -k 10 300 python tools/probe/ntt_ab.py 2 abtest/lib_ntt_A.so abtest/lib_ntt_E.so abtest/lib_ntt_F.so > gpurun_out/ntt_ab2.txt 2>&1
bash tools/gpu/r2_ntt_pmc.sh abtest/lib_ntt_A.so abtest/lib_ntt_E.so
