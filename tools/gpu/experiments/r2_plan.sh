# Isolated H-plan sort timing + per-kernel stats, then the sort parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "dense or msm" --timeout 200 --timeout-method thread > gpurun_out/gt_plan.log 2>&1
timeout -k 10 300 python3 tools/probe/plan_bench.py 23 10 > gpurun_out/plan.json 2> gpurun_out/plan.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_plan -o run -- python3 tools/probe/plan_bench.py 23 5 > gpurun_out/prof_plan.log 2>&1
