# Batch scheduler check: its GPU tests, then the bench with the PCIe-inclusive batch line.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prove.py tests/test_node.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gt_batch.log 2>&1
timeout -k 10 400 python bench.py --cpu-baseline none > gpurun_out/bench_batch.log 2>&1
