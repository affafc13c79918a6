# round 5: kernel-level MSMs with the H plan's 48-entry tasks: the kernel / proof GPU tests and the
# default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f5
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
