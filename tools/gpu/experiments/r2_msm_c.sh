# configs[1] G1 MSM 2^20: window bits x plan (compacted rocprim / dense hand-sorted) sweep
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/msm_c.txt
for d in 0 1; do for c in 16 17 18 19 20; do
  echo "dense=$d c=$c $(ZKP_MSM_DENSE=$d ZKP_MSM_C=$c timeout -k 10 120 python3 tools/probe/msm_run.py 20 | tail -1)" >> gpurun_out/msm_c.txt
done; done
