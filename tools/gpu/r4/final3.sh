# round 4, last check with the three-class witness transfer: the whole GPU suite, smoke(), the default
# bench line, and the same bench under rocprofv3 --kernel-trace --marker-trace with the per-launch split
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_final3.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_final3.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_final3.json 2> gpurun_out/r4/bench_final3.err
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r4/prof9 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r4/bench_prof9.json 2> gpurun_out/r4/bench_prof9.err
python3 tools/prof/launch_split.py gpurun_out/r4/prof9/run_kernel_trace.csv gpurun_out/r4/prof9/run_marker_api_trace.csv gpurun_out/r4/bench_prof9.json gpurun_out/r4/launch_split9.json > /dev/null
