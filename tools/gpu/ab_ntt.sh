# lazy radix-4 NTT sums: GPU NTT/prove tests, then A/B vs lib/libzkp_amd_base.so (bench with kernel lines)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=zk-p2p-onramp_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
cp $L/libzkp_amd.so /tmp/new.so
for v in new base new base; do
  if [ $v = base ]; then cp $L/libzkp_amd_base.so $L/libzkp_amd.so; else cp /tmp/new.so $L/libzkp_amd.so; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none >> gpurun_out/bn_$v.log 2>&1
done
cp /tmp/new.so $L/libzkp_amd.so
