set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 6 --warmup 2 --cpu-baseline none > gpurun_out/b1.log 2>&1
ZKP_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 --cpu-baseline none > gpurun_out/b2.log 2>&1
