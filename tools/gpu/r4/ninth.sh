# round 4, ninth call: witness expansion per chunk behind its DMA (lib_perchunk) vs one expansion at
# the end (in-tree): transfer tests, then the latency probe alternating, 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_perchunk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_perchunk.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_base_$i.txt 2> gpurun_out/r4/lat_base_$i.err
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_perchunk.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_pc_$i.txt 2> gpurun_out/r4/lat_pc_$i.err
done
