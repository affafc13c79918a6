# round 5: accumulate task sizes re-measured on the round-5 kernels (rounds 2-3 chose 32 for both plans):
# the short staged bench with ZKP_MSM task_h / task_w overrides, alternated 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/r5/ab.sh 3 task "base:-" "th24:ZKP_MSM=task_h=24" "th48:ZKP_MSM=task_h=48" "th64:ZKP_MSM=task_h=64" "tw64:ZKP_MSM=task_w=64"
echo ab done
