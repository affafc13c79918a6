# split proof (configs[4], S24): distributed vs recomputed quotient, slices emulated on one GPU
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 200 > gpurun_out/gts.log 2>&1
timeout -k 10 500 python bench.py --mode split --parts 2 --quotient dist --steps 4 --warmup 1 > gpurun_out/bs_dist.log 2>&1
timeout -k 10 500 python bench.py --mode split --parts 2 --quotient full --steps 4 --warmup 1 > gpurun_out/bs_full.log 2>&1
