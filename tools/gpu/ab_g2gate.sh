# G2 finish gated on the H plan (ZKP_G2_FINISH_GATE=2: on the high-priority stream s3) vs ungated
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ZKP_G2_FINISH_GATE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py tests/test_gpu_split.py -x -q --timeout 200 > gpurun_out/gt_g2gate.log 2>&1
for g in 2 0 2 0 2 0; do
  ZKP_G2_FINISH_GATE=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bg_$g.log 2>&1
done
ZKP_G2_FINISH_GATE=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_g2gate -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/pg.log 2>&1
