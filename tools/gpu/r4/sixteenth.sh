# round 4, sixteenth call: three-class witness encoding (bit values in the block metadata) and an empty
# kernel on each compute stream at the start of a host-witness proof ("prewarm"): transfer tests, then
# the latency probe over the 2 x 2 variants, alternating, 2 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_3c.log 2>&1
L=$PWD/tools/gpu/r4/libs
for i in 1 2; do
  ZKP_LIB_PATH=$L/lib_head.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_head_$i.txt 2> gpurun_out/r4/lat_head_$i.err
  ZKP_LIB_PATH=$L/lib_prewarm.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_pw_$i.txt 2> gpurun_out/r4/lat_pw_$i.err
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_3c_$i.txt 2> gpurun_out/r4/lat_3c_$i.err
  ZKP_LIB_PATH=$L/lib_3c_pw.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_3cpw_$i.txt 2> gpurun_out/r4/lat_3cpw_$i.err
done
