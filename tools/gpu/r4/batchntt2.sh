# round 4: the split quotient stage batched, the proof's per-vector (kept): parity tests + default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_split.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/batchntt2_tests.txt 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/r4/batchntt2_bench.json 2> gpurun_out/r4/batchntt2_bench.err
