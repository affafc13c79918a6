# round 4: batched coset extension (A, B, C one launch per pass): parity tests of the quotient paths,
# the per-vector NTT times, then the default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_split.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/batchntt_tests.txt 2>&1
timeout -k 10 180 python3 tools/probe/ntt_batch.py 2 > gpurun_out/r4/ntt_batch.txt 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/r4/batchntt_bench.json 2> gpurun_out/r4/batchntt_bench.err
