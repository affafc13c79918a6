# round 5: the bucket-reduction segment (M buckets per running-sum segment, default 4) re-measured with the
# round-5 finish: seg 2 / 8 vs 4, alternated 3 rounds on the short staged bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/r5/ab.sh 3 seg "base:-" "seg2:ZKP_MSM=seg=2" "seg8:ZKP_MSM=seg=8"
echo ab done
