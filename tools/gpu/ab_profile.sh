# A/B kernel traces on one box: serial breakdown and concurrent timeline for the base library
# (abtest/libzkp_amd_base.so) and the in-tree one.  Summaries only (raw traces stay on the box).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0"
W=/tmp/zkp_ab
for v in base new; do
  rm -rf $W && mkdir -p $W
  if [ $v = base ]; then export ZKP_LIB_PATH=$PWD/abtest/libzkp_amd_base.so; else unset ZKP_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/conc -o run -- $B > gpurun_out/ab/conc_$v.log 2>&1
  ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/ser -o run -- $B > gpurun_out/ab/ser_$v.log 2>&1
  cp $W/conc/run_kernel_stats.csv gpurun_out/ab/conc_stats_$v.csv
  (cd tools/prof && python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/ab/timeline_$v.txt && python3 breakdown.py $W/ser/run_kernel_stats.csv > ../../gpurun_out/ab/serial_$v.txt)
done
rm -rf $W
