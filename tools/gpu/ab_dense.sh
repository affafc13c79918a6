# dense H plan (default) vs compacted (ZKP_H_DENSE=0): GPU suite, A/B bench, concurrent trace
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1
for d in 1 0 1 0; do
  ZKP_H_DENSE=$d timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bd_$d.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/pc.log 2>&1
