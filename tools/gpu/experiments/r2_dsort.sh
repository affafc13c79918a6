# Dense-plan counting sort: GPU parity, bench A/B against the rocprim radix sort, concurrent trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gt_dsort.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline none > gpurun_out/b_dsort.log 2>&1
ZKP_H_SORT=rocprim timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_rocprim.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/prof_conc.log 2>&1
