# configs[1] G1 MSM 2^20 pipeline breakdown: rocprofv3 kernel stats, compacted (rocprim) vs dense plan
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/msm20
for d in 0 1; do
  ZKP_MSM_DENSE=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/msm20/dense$d -o run --output-format csv -- python3 tools/probe/msm_run.py 20 > gpurun_out/msm20/dense$d.log 2>&1
done
