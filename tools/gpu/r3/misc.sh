# round 3: the concurrent-staged test, configs[4] S24 split over 8 balanced slices on one GPU at HEAD,
# and verify-before-return in the batch line (host pairing of proof i beside proof i+1's device work)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py -x -q --timeout 200 --timeout-method thread -k "staged_concurrent or inflight" > gpurun_out/gt_misc.log 2>&1
ZKP_SPLIT_BALANCE=1 timeout -k 10 600 python bench.py --mode split --parts 8 --steps 2 --warmup 1 > gpurun_out/split8_r3.log 2>&1
ZKP_VERIFY=1 timeout -k 10 300 python bench.py --steps 8 --cpu-baseline none --no-kernels --batch 64 > gpurun_out/verify_batch_r3.log 2>&1
