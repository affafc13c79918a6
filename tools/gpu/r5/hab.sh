# round 5: H window bits 20 (default) vs 22 (12 windows instead of 13: -7.7 % additions, 4x the buckets),
# alternated, 3 rounds; then the default bench once with the two-in-flight side line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/r5/ab.sh 3 h22 "h20:-" "h22:ZKP_MSM=h=22"
echo ab done
timeout -k 10 500 python bench.py > gpurun_out/r5/bench_b.json 2> gpurun_out/r5/bench_b.err
echo bench done
