# round 4, third call: GPU suite (compact witness transfer), smoke, the default bench line, and the
# same bench under rocprofv3 --kernel-trace --marker-trace for the per-launch split
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_prove.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_third.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_third.json 2> gpurun_out/r4/bench_third.err
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r4/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r4/bench_prof.json 2> gpurun_out/r4/bench_prof.err
python3 tools/prof/launch_split.py $(ls gpurun_out/r4/prof/*kernel_trace.csv | head -1) $(ls gpurun_out/r4/prof/*marker_api_trace.csv | head -1) gpurun_out/r4/bench_prof.json gpurun_out/r4/launch_split.json > /dev/null
