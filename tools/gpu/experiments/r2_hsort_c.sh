# dense plan at c = 18 / 19 / 20 (2^20 MSM): which kernel is slow at 18 and 19
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hsc
for c in 18 19 20; do
  ZKP_MSM_C=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hsc/c$c -o run --output-format csv -- python3 tools/probe/msm_run.py 20 > gpurun_out/hsc/c$c.log 2>&1
done
