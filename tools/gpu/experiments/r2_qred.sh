# qreduce check: field/NTT/MSM/prove GPU tests, then a bench without the CPU baseline.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or quotient or msm or prove or golden or smoke" > gpurun_out/qred_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 > gpurun_out/qred_bench.log 2>&1
