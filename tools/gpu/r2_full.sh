# Full GPU suite + default bench (no CPU baseline) + isolated accumulate/NTT kernels line.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt_full.log 2>&1
timeout -k 10 400 python bench.py --cpu-baseline none > gpurun_out/b_full.log 2>&1
