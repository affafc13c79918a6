# round 4, seventh call:
# the whole GPU suite, smoke, the latency probe with the witness file
# mapped (zkp_prove_files) vs read into a buffer, the default bench line, and the same bench under
# rocprofv3 --kernel-trace --marker-trace with the per-launch split
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gt_seventh.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_seventh.log 2>&1
ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_readfile.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/latency_readfile.txt 2> gpurun_out/r4/latency_readfile.err
timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/latency_mmap.txt 2> gpurun_out/r4/latency_mmap.err
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_seventh.json 2> gpurun_out/r4/bench_seventh.err
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r4/prof7 -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > gpurun_out/r4/bench_prof7.json 2> gpurun_out/r4/bench_prof7.err
python3 tools/prof/launch_split.py gpurun_out/r4/prof7/run_kernel_trace.csv gpurun_out/r4/prof7/run_marker_api_trace.csv gpurun_out/r4/bench_prof7.json gpurun_out/r4/launch_split7.json > /dev/null
