# the default bench timing loop under rocprofv3 --kernel-trace --marker-trace --stats, then the per-launch
# split of the accumulate launches (tools/prof/launch_split.py; profiles/launch_split_r0N.json)
#   bash tools/gpu/trace.sh <tag>  ->  $O/prof/run_*.csv, $O/bench_prof.json, $O/launch_split.json
source "$(dirname "$0")/common.sh"
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0 > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/launch_split.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/bench_prof.json $O/launch_split.json > /dev/null
echo trace done
