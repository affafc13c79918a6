set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_kernels.py -x -q --timeout 200 > gpurun_out/gt.log 2>&1
timeout -k 10 400 python bench.py --mode split --parts 2 --steps 2 --warmup 1 > gpurun_out/bsplit.log 2>&1
