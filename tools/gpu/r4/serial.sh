# round 4: every kernel of a proof alone (ZKP_SERIAL=1), kernel trace: the H accumulation's time
# without the G2 finish beside it
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/r4/serial -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r4/serial.json 2> gpurun_out/r4/serial.err
