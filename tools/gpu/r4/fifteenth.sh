# round 4, fifteenth call: what the idle-gap penalty is made of (latency probe gap modes); 8 vs 4 copy
# queues for the witness transfer
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
LATENCY_PROBE_GAP_MODES=1 timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_gapmodes.txt 2> gpurun_out/r4/lat_gapmodes.err
for i in 1 2; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_dma8.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_dma8_$i.txt 2> gpurun_out/r4/lat_dma8_$i.err
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_dma4b_$i.txt 2> gpurun_out/r4/lat_dma4b_$i.err
done
