# round 3, first call: H window-bits sweep (16/17 vs 20), then the multi-device bench path
# (--gpus 2 on a 1-GPU box must fail with status 2; --gpus 2 --rehearsal runs 2 logical devices)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/hsweep.txt
bash tools/gpu/experiments/r2_hsweep17.sh
set +e
timeout -k 10 120 python bench.py --gpus 2 --cpu-baseline none > gpurun_out/r3_gpus2.log 2>&1
echo "gpus2 rc=$?" >> gpurun_out/hsweep.txt
set -e
timeout -k 10 300 python bench.py --gpus 2 --rehearsal --steps 8 --warmup 2 --cpu-baseline none --no-kernels --batch 32 > gpurun_out/r3_rehearsal.log 2>&1
tail -1 gpurun_out/r3_rehearsal.log >> gpurun_out/hsweep.txt
