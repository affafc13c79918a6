# automatic dense window bits at 2^21 / 2^22 points: base library vs the top-window-aware choice
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/hsc3.txt
for k in 21 22; do
  for lib in abtest/libzkp_amd_base.so zk-p2p-onramp_amd/lib/libzkp_amd.so; do
    echo "2^$k $lib $(ZKP_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 tools/probe/msm_run.py $k | tail -1)" >> gpurun_out/hsc3.txt
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "msm" > gpurun_out/hsc3_tests.log 2>&1
