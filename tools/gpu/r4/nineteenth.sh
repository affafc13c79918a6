# round 4, nineteenth call: the idle-gap penalty with every other host core busy, and with 4-KB memsets through the gap
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
LATENCY_PROBE_GAP_MODES=1 timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_gapmodes3.txt 2> gpurun_out/r4/lat_gapmodes3.err
