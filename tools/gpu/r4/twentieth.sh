# round 4, twentieth call: kernel trace of the latency probe (back-to-back vs gapped staged proofs)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/gaptrace -o run -- python3 tools/probe/latency_probe.py > gpurun_out/r4/gaptrace.txt 2> gpurun_out/r4/gaptrace.err
