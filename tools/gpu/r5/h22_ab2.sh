# round 5: H window 22 again, now that H tasks hold 48 entries: at c = 22 a bucket holds ~48 entries, one
# task and no merge; h20 (default) vs h22 vs h22 with 64-entry tasks, alternated 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/r5/ab.sh 3 h22b "base:-" "h22:ZKP_MSM=h=22" "h22t64:ZKP_MSM=h=22,task_h=64"
echo ab done
