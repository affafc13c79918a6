# round 4: the default bench line as the driver runs it
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_default.json 2> gpurun_out/r4/bench_default.err
