# round 5, final library (NTT w^0 step, H-plan tasks of 48; bench with the frozen Python heap): the whole GPU suite, smoke(),
# the default bench line, and the same bench under rocprofv3 --kernel-trace --marker-trace --stats with
# the per-launch split and the batch/staged split
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gt_final.log 2>&1
echo suite done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 64 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/launch_split.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/bench_prof.json $O/launch_split.json > /dev/null
python3 tools/prof/batch_gaps.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/batch_gaps.json > /dev/null
echo trace done
