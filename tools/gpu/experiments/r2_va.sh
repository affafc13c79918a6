# one-ahead index load in the accumulate + shorter chain level below the subset trees: MSM tests, A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msm or golden or fullsize" > gpurun_out/va_tests.log 2>&1
timeout -k 10 300 python tools/probe/msm_ab.py 2 abtest/libzkp_amd_base.so abtest/lib_va.so > gpurun_out/va_msm_ab.txt 2>&1
bash tools/gpu/ab.sh 3
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
