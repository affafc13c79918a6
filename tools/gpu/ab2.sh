# A/B: new lib (default) vs lib/libzkp_amd_base.so, plus H-plan window bits 22; GPU MSM tests first
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=zk-p2p-onramp_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 200 > gpurun_out/gt.log 2>&1
cp $L/libzkp_amd.so /tmp/new.so
for v in new base new base; do
  cp $L/libzkp_amd_$v.so $L/libzkp_amd.so 2>/dev/null || cp /tmp/new.so $L/libzkp_amd.so
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/ab_$v.log 2>&1
done
cp /tmp/new.so $L/libzkp_amd.so
for h in 22 20 22; do
  ZKP_WINDOW_BITS_H=$h timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bh_$h.log 2>&1
done
