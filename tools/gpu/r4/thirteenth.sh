# round 4, thirteenth call: memory-copy + kernel trace of the latency probe (where the witness
# transfer's time goes: DMA count and gaps)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4/lattrace -o run -- python3 tools/probe/latency_probe.py > gpurun_out/r4/lattrace.txt 2> gpurun_out/r4/lattrace.err
