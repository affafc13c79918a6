# round 5: where the batch line loses ~5 % against the staged headline: the bench (staged loop + a
# 64-proof batch from host memory) under rocprofv3 --kernel-trace --marker-trace; tools/prof/batch_gaps.py
# splits the trace by the "bench timed" / "batch timed" ROCTx ranges.  Plus the new NTT geometry tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/bt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "ntt" > $O/gt_ntt.log 2>&1
echo gt done
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 64 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/batch_gaps.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/batch_gaps.json > /dev/null
echo trace done
