# round 3: the whole GPU suite, smoke, the default bench line and the all-uniform-witness line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gt_full_r3.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r3.json 2> gpurun_out/bench_r3.err
timeout -k 10 300 python bench.py --bool-pct 0 --cpu-baseline none --batch 64 > gpurun_out/bench_r3_bool0.json 2> gpurun_out/bench_r3_bool0.err
