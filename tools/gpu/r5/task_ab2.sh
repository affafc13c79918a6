# round 5: H-plan task size follow-up (task_h=48 led base in 3 of 3 rounds by +0.1 to +1.5 %): base (32),
# 40, 48, 56, alternated 4 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/r5/ab.sh 4 task2 "base:-" "th40:ZKP_MSM=task_h=40" "th48:ZKP_MSM=task_h=48" "th56:ZKP_MSM=task_h=56"
echo ab done
