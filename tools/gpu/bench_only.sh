set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-baseline none > gpurun_out/b.log 2>&1
