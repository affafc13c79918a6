# A/B of two builds of libzkp_amd.so: lib/libzkp_amd.so (A) vs lib/libzkp_amd_$1.so (B)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -q --timeout 200 > gpurun_out/gt.log 2>&1
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels"
for v in A B; do
  if [ $v = B ]; then cp zk-p2p-onramp_amd/lib/libzkp_amd_$1.so zk-p2p-onramp_amd/lib/libzkp_amd.so; fi
  timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/ab_$v.log 2>&1
  ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_prof_$v -o run -- $B > gpurun_out/ab_p$v.log 2>&1
done
