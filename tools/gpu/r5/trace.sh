# round 5: (1) the default bench command under rocprofv3 --kernel-trace --marker-trace --stats: the
# per-launch split of the accumulate launches (tools/prof/launch_split.py) and the kernel summary for
# profiles/; (2) VERDICT r4 item 4, the host side of configs[3] at N = 8 on this box's host cores: the
# encoder probe (8 groups = 8 devices, the Venmo 70 % mix and the all-uniform mix, 16 and 2 threads per
# group) and one bench.py --gpus 8 --rehearsal line (8 pipelines' worth of host threads on GPU 0)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
mkdir -p $O
# host-witness latency, round-4 library vs this one, alternated (the bench line moved 27.5 -> 29.4 ms)
for i in 1 2; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_base_$i.txt 2> $O/lat_base_$i.err
  timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_cur_$i.txt 2> $O/lat_cur_$i.err
done
echo latency done
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/launch_split.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/bench_prof.json $O/launch_split.json > /dev/null
echo trace done
for pct in 70 0; do
  for t in 16 4 2; do
    timeout -k 10 60 tools/hosttest/host_capacity_bin 6400562 8 $t 8 $pct 2 >> $O/host_capacity.txt 2>&1
  done
  timeout -k 10 60 tools/hosttest/host_capacity_bin 6400562 1 16 5 $pct 2 >> $O/host_capacity.txt 2>&1
done
echo probe done
timeout -k 10 900 python3 bench.py --gpus 8 --rehearsal --no-kernels --cpu-baseline none --no-bool0-line > $O/rehearsal8.json 2> $O/rehearsal8.err
echo rehearsal done
