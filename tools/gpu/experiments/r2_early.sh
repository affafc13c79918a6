# early host blinding (A, B, C-partial while the H MSM runs): proof GPU tests, proof A/B, boundary timeline
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prove or golden or batch or split or node or random or calldata" > gpurun_out/early_tests.log 2>&1
bash tools/gpu/ab.sh 2
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
W=/tmp/zkp_prof; rm -rf $W && mkdir -p $W
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $W/conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0 > gpurun_out/prof/conc3.log 2>&1
(cd tools/prof && python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/prof/timeline3.txt)
rm -rf $W
