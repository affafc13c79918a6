# round 4, final check: the whole GPU suite, smoke(), the default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_final.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_final.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_final.json 2> gpurun_out/r4/bench_final.err
