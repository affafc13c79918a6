# round 4, first check after pruning the knobs: GPU suite, smoke(), the default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_first.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_first.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_first.json 2> gpurun_out/r4/bench_first.err
timeout -k 10 300 tools/ubench/acc_bench 19 208 5 > gpurun_out/r4/acc_bench_first.txt 2>&1
