# round 3 check at HEAD: the whole GPU suite, smoke(), the default bench line (CPU baseline and
# batch line included), the all-uniform-witness line and the verify-before-return cost
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt_final_r3.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final_r3.log 2>&1
timeout -k 10 500 python bench.py > gpurun_out/bench_final_r3.json 2> gpurun_out/bench_final_r3.err
timeout -k 10 300 python bench.py --bool-pct 0 --cpu-baseline none --batch 64 > gpurun_out/bench_final_r3_bool0.json 2> gpurun_out/bench_final_r3_bool0.err
ZKP_VERIFY=1 timeout -k 10 300 python bench.py --steps 8 --cpu-baseline none --batch 0 --no-kernels > gpurun_out/bench_final_r3_verify.json 2> gpurun_out/bench_final_r3_verify.err
