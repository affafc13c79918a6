# round 4, fourteenth call: witness-transfer copies over 1 / 2 (in-tree) / 4 copy queues: transfer
# tests, then the latency probe alternating (3 rounds), then one copy trace with 2 queues
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_dma2.log 2>&1
ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_dma4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_dma4.log 2>&1
for i in 1 2 3; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_dma1.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_dma1_$i.txt 2> gpurun_out/r4/lat_dma1_$i.err
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_dma2_$i.txt 2> gpurun_out/r4/lat_dma2_$i.err
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_dma4.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_dma4_$i.txt 2> gpurun_out/r4/lat_dma4_$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4/lattrace2 -o run -- python3 tools/probe/latency_probe.py > gpurun_out/r4/lattrace2.txt 2> gpurun_out/r4/lattrace2.err
