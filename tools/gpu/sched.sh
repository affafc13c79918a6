set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py tests/test_gpu_split.py -x -q --timeout 200 > gpurun_out/gt.log 2>&1
for g in 1 0; do
  ZKP_SCHED=$g timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_g$g.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/pc.log 2>&1
