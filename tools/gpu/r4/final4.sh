# round 4, last check with the batched split-stage NTT: the whole GPU suite, smoke(), the default
# bench line, and the same bench under rocprofv3 --kernel-trace --marker-trace with the per-launch split
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_final4.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_final4.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_final4.json 2> gpurun_out/r4/bench_final4.err
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r4/prof10 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r4/bench_prof10.json 2> gpurun_out/r4/bench_prof10.err
python3 tools/prof/launch_split.py gpurun_out/r4/prof10/run_kernel_trace.csv gpurun_out/r4/prof10/run_marker_api_trace.csv gpurun_out/r4/bench_prof10.json gpurun_out/r4/launch_split10.json > /dev/null
