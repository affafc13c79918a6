# split-proof balance: GPU split tests (incl. ZKP_SPLIT_BALANCE=1 cases), then S24 in 8 slices with balance
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1
ZKP_SPLIT_BALANCE=1 timeout -k 10 900 python bench.py --mode split --parts 8 --steps 2 --warmup 1 > gpurun_out/split8_bal.log 2>&1
