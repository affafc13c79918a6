# round 4, sixth call: per-chunk witness expansion (tests + latency probe), and the batch line with
# 16 encode threads always vs a quarter of them beside a proof in flight (A/B, 2 rounds)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_sixth.log 2>&1
timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/latency_probe_6.txt 2> gpurun_out/r4/latency_probe_6.err
for i in 1 2; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_up16.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/ab_up_base_$i.json 2> gpurun_out/r4/ab_up_base_$i.err
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/ab_up_new_$i.json 2> gpurun_out/r4/ab_up_new_$i.err
done
