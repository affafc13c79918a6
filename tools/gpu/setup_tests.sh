set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_setup_contrib.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/gt_setup.log 2>&1
timeout -k 10 300 python tools/bench_setup.py > gpurun_out/bench_setup.log 2>&1
