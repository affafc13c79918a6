# round 4, twenty-first call: a clock warm-up kernel (full VALU load, 2048 x 256 lanes) on the G2
# stream at the start of a host-witness proof, during the transfer: 3000 / 6000 iterations vs none,
# latency probe alternating, 2 rounds; one kernel trace of the 6000 variant
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
L=$PWD/tools/gpu/r4/libs
for i in 1 2; do
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_nowarm_$i.txt 2> gpurun_out/r4/lat_nowarm_$i.err
  ZKP_LIB_PATH=$L/lib_warm3000.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_warm3000_$i.txt 2> gpurun_out/r4/lat_warm3000_$i.err
  ZKP_LIB_PATH=$L/lib_warm6000.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_warm6000_$i.txt 2> gpurun_out/r4/lat_warm6000_$i.err
done
ZKP_LIB_PATH=$L/lib_warm6000.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/warmtrace -o run -- python3 tools/probe/latency_probe.py > gpurun_out/r4/warmtrace.txt 2> gpurun_out/r4/warmtrace.err
