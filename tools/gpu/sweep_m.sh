# bucket-reduction segment size M and subset fan-in L (ZKP_SEG_M / ZKP_SUB_L)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ZKP_SEG_M=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py -x -q --timeout 200 > gpurun_out/gt_m16.log 2>&1
for rep in 1 2; do
  for cfg in "4 8" "8 8" "16 8" "32 8" "16 4" "16 16"; do
    set -- $cfg
    ZKP_SEG_M=$1 ZKP_SUB_L=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bm_$1_$2.log 2>&1
  done
done
