# bucket binning plan vs the rocprim radix-sort plan: GPU tests, bench, serial + concurrent traces
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 > gpurun_out/gt.log 2>&1
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels"
for m in bins radix bins radix; do
  ZKP_PLAN_SORT=$m timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bb_$m.log 2>&1
done
ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o run -- $B > gpurun_out/bp4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_conc -o run -- $B > gpurun_out/pc.log 2>&1
