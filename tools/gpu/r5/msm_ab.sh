# round 5: the configs[1] G1 MSM 2^20 with 48-entry tasks (the H plan's new size) vs 32, alternated 4 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5 && timeout -k 10 600 python3 tools/probe/msm_ab.py 4 "task_h=32" "-" "task_h=64" > gpurun_out/r5/msm_ab.txt 2>&1
cat gpurun_out/r5/msm_ab.txt
