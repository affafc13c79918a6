# Round-2 check at HEAD: full GPU suite, smoke(), default bench (CPU baseline included)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt_final.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/b_final.log 2>&1
