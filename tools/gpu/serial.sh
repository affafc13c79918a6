# tests + bench + serial (one kernel at a time) kernel profile
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 200 > gpurun_out/gt.log 2>&1
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b.log 2>&1
ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/bp4.log 2>&1
